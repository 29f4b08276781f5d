#!/usr/bin/env python3
"""Per-phase wall-cycle shares of k_decode_pp (diagnostic build).

    make -C bo-lz4-ada_amd/csrc variant NAME=ppst DEFS=-DLZ4ADA_PP_STAMPS
    python tools/pp_stamps.py --kinds mixed,dense
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("LZ4ADA_LIB", os.path.join(ROOT, "bo-lz4-ada_amd", "_variants",
                                                  "liblz4ada_hip_ppst.so"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import lz4ada  # noqa: E402

NAMES = ["PASS1", "WSTAGED", "STAGE", "CUT", "PRE", "HBMW", "LIT", "TOKW", "RING", "FLUSH", "OVER",
         "TAIL", "BATCHES", "WAVES"]
COUNTS = {"BATCHES", "WAVES"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", default="mixed")
    ap.add_argument("--blocks", type=int, default=2048)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    bmax = 4 << 20
    f = lz4ada._lib.lz4ada_pp_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * len(NAMES))()
    import lz4frame
    import xxhash
    for kind in args.kinds.split(","):
        recs = bench.make_unique_blocks(lz4ada, lz4frame, xxhash, kind, 16, bmax)
        fr, fl, de, eh, cb, rb, _ = bench.assemble_shard(lz4ada, torch, recs, 0, args.blocks, bmax, dev)
        out = torch.empty(args.blocks * bmax, dtype=torch.uint8, device=dev)
        st = torch.zeros(args.blocks * 32, dtype=torch.uint8, device=dev)
        sh = torch.cuda.current_stream(dev).cuda_stream
        lz4ada.launch_decode_variant(fr.data_ptr(), fl, de.data_ptr(), args.blocks, out.data_ptr(),
                                     st.data_ptr(), lz4ada.DECODE_PP_ALONE, sh)
        torch.cuda.synchronize()
        f(buf, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lz4ada.launch_decode_variant(fr.data_ptr(), fl, de.data_ptr(), args.blocks, out.data_ptr(),
                                     st.data_ptr(), lz4ada.DECODE_PP_ALONE, sh)
        e1.record()
        torch.cuda.synchronize()
        f(buf, 1)
        v = dict(zip(NAMES, list(buf)))
        waves = max(v["WAVES"], 1)
        print(f"== {kind}: {e0.elapsed_time(e1):.3f} ms; per wave (Mcycles, s_memtime), "
              f"{v['BATCHES'] / waves:.0f} batches per wave")
        # pass 1 is summed over both waves of each block
        print(f"  {'PASS1':8s} {v['PASS1'] / waves / 1e6:8.3f}")
        tot = sum(v[k] for k in NAMES if k not in COUNTS and k != "PASS1")
        for k in NAMES:
            if k in COUNTS or k == "PASS1":
                continue
            print(f"  {k:8s} {v[k] / waves / 1e6:8.3f}  {100 * v[k] / max(tot, 1):5.1f}%")
        print(f"  {'pass 2':8s} {tot / waves / 1e6:8.3f}")
        del fr, de, out, st


if __name__ == "__main__":
    main()
