#!/usr/bin/env python3
"""HBM-sourced match gathers of k_decode_idx on the bench workload
(diagnostic build, VERDICT r4 item 6: where FETCH_SIZE goes).

    make -C bo-lz4-ada_amd/csrc variant NAME=gath DEFS=-DLZ4ADA_IDX_GATHERS
    python tools/gathers.py --kinds mixed,dense
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("LZ4ADA_LIB", os.path.join(ROOT, "bo-lz4-ada_amd", "_variants",
                                                  "liblz4ada_hip_gath.so"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import lz4ada  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", default="mixed")
    ap.add_argument("--blocks", type=int, default=2048)
    ap.add_argument("--real", default="", help="t1111k,liblz4_text: encoder blocks (bench.real_sources)")
    args = ap.parse_args()
    import lz4frame
    import xxhash
    f = lz4ada._lib.lz4ada_idx_gathers
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 4)()
    dev = torch.device("cuda", 0)
    bmax = 4 << 20
    for kind in (args.real.split(",") if args.real else args.kinds.split(",")):
        recs = (bench.real_sources(kind)[0] if args.real else
                bench.make_unique_blocks(lz4ada, lz4frame, xxhash, kind, 64, bmax))
        fr, fl, de, eh, cb, rb, _ = bench.assemble_shard(lz4ada, torch, recs, 0, args.blocks, bmax, dev)
        out = torch.empty(args.blocks * bmax, dtype=torch.uint8, device=dev)
        st = torch.zeros(args.blocks * 32, dtype=torch.uint8, device=dev)
        sh = torch.cuda.current_stream(dev).cuda_stream
        f(buf, 1)  # reset (what an earlier launch left)
        lz4ada.launch_decode_variant(fr.data_ptr(), fl, de.data_ptr(), args.blocks, out.data_ptr(),
                                     st.data_ptr(), lz4ada.DECODE_IDX1_ALONE, sh)
        torch.cuda.synchronize()
        f(buf, 1)  # this launch's counts
        loads, touches, batches, _ = list(buf)
        print(f"== {kind}: {args.blocks} blocks, {cb / 1e9:.2f} GB in, {rb / 1e9:.2f} GB out; "
              f"HBM-sourced match loads {loads / 1e6:.1f} M = {16 * loads / 1e9:.2f} GB requested, "
              f"{touches / 1e6:.1f} M line touches = {128 * touches / 1e9:.2f} GB at 128 B/line, "
              f"{64 * touches / 1e9:.2f} GB at 64 B; {batches / args.blocks:.0f} batches per block with one")
        del fr, de, out, st


if __name__ == "__main__":
    main()
