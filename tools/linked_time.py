#!/usr/bin/env python3
"""configs[4]'s linked row alone (bench.bench_linked: 4096 x 256 KiB mixed
blocks, device-resident) and its phase times (LZ4ADA_TRACE_LINKED=1 prints
them to stderr)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))

import torch  # noqa: E402
import xxhash  # noqa: E402

import bench  # noqa: E402
import lz4ada  # noqa: E402
import lz4frame  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    st = torch.cuda.current_stream(dev)
    kind = sys.argv[1] if len(sys.argv) > 1 else "mixed"
    r = bench.bench_linked((lz4ada, lz4frame, xxhash, torch), dev, st.cuda_stream, st, kind=kind)
    print(json.dumps({k: r[k] for k in ("decode_ms", "MiB_s", "frac")}), kind, flush=True)
