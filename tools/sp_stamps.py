#!/usr/bin/env python3
"""Phase cycles of k_decode_sparse (diagnostic build):

    make -C bo-lz4-ada_amd/csrc variant NAME=spst DEFS=-DLZ4ADA_SP_STAMPS
    python tools/sp_stamps.py --kind literal
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("LZ4ADA_LIB", os.path.join(ROOT, "bo-lz4-ada_amd", "_variants",
                                                  "liblz4ada_hip_spst.so"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import lz4ada  # noqa: E402

NAMES = ["SP_TOTAL", "SP_DMAWAIT", "SP_MWAIT", "SP_MATCH", "SP_GCOPY", "SP_BATCHES", "SP_RESTARTS",
         "SP_SEQ", "SP_SLOW"]
COUNTS = {"SP_BATCHES", "SP_RESTARTS", "SP_SEQ", "SP_SLOW"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="literal")
    ap.add_argument("--blocks", type=int, default=2048)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    bmax = 4 << 20
    f = lz4ada._lib.lz4ada_sp_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * len(NAMES))()
    import lz4frame
    import xxhash
    recs = bench.make_unique_blocks(lz4ada, lz4frame, xxhash, args.kind, 16, bmax)
    fr, fl, de, eh, cb, rb, _ = bench.assemble_shard(lz4ada, torch, recs, 0, args.blocks, bmax, dev)
    out = torch.empty(args.blocks * bmax, dtype=torch.uint8, device=dev)
    st = torch.zeros(args.blocks * 32, dtype=torch.uint8, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    for rep in range(2):
        f(buf, 1)
        lz4ada.launch_decode_variant(fr.data_ptr(), fl, de.data_ptr(), args.blocks, out.data_ptr(),
                                     st.data_ptr(), lz4ada.DECODE_IDX_SPARSE, sh)
        torch.cuda.synchronize()
    f(buf, 1)
    v = dict(zip(NAMES, list(buf)))
    nb = args.blocks
    tot = max(v["SP_TOTAL"], 1)
    print(f"== {args.kind}: per block, {cb / nb / 1024:.0f} KiB in, {rb / nb / 1024:.0f} KiB out")
    for k in NAMES:
        if k in COUNTS:
            print(f"   {k:12s} {v[k] / nb:14.1f}")
        else:
            print(f"   {k:12s} {v[k] / nb:14.0f}  {100 * v[k] / tot:5.1f}%")


if __name__ == "__main__":
    main()
