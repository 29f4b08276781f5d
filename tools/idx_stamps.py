#!/usr/bin/env python3
"""Per-phase cycle shares of k_index / k_decode_idx (diagnostic build).

    make -C bo-lz4-ada_amd/csrc variant NAME=idxst DEFS=-DLZ4ADA_IDX_STAMPS
    python tools/idx_stamps.py --kind mixed
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("LZ4ADA_LIB", os.path.join(ROOT, "bo-lz4-ada_amd", "_variants",
                                                  "liblz4ada_hip_idxst.so"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import bench  # noqa: E402
import lz4ada  # noqa: E402

NAMES = ["I_STAGE", "I_WALK0", "I_ITER", "I_CHUNKS", "I_ITERS",
         "D_STAGE", "D_WALK1", "D_WALK2", "D_TLDS", "D_LIT", "D_MFAR", "D_NEAR", "D_FLUSH", "D_GLOBAL",
         "D_BATCHES", "D_GBATCHES", "D_ROUNDS", "D_TASKS", "D_LANES", "I_STEPS", "I_MAXST"]
COUNTS = {"I_CHUNKS", "I_ITERS", "D_BATCHES", "D_GBATCHES", "D_ROUNDS", "D_TASKS", "D_LANES",
          "I_STEPS", "I_MAXST"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", default="mixed")
    ap.add_argument("--blocks", type=int, default=2048)
    ap.add_argument("--block-max", type=int, default=4 << 20)
    ap.add_argument("--real", default="", help="t1111k / liblz4_text: encoder blocks (bench.real_sources)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    bmax = args.block_max
    f = lz4ada._lib.lz4ada_idx_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * len(NAMES))()
    for kind in ([args.real] if args.real else args.kinds.split(",")):
        import lz4frame
        import xxhash
        recs = (bench.real_sources(kind)[0] if args.real else
                bench.make_unique_blocks(lz4ada, lz4frame, xxhash, kind, 64, bmax))
        fr, fl, de, eh, cb, rb, _ = bench.assemble_shard(lz4ada, torch, recs, 0, args.blocks, bmax,
                                                         dev)
        out = torch.empty(args.blocks * bmax, dtype=torch.uint8, device=dev)
        st = torch.zeros(args.blocks * 32, dtype=torch.uint8, device=dev)
        sh = torch.cuda.current_stream(dev).cuda_stream
        f(buf, 1)
        lz4ada.launch_decode_variant(fr.data_ptr(), fl, de.data_ptr(), args.blocks, out.data_ptr(),
                                     st.data_ptr(), lz4ada.DECODE_IDX_ALONE, sh)
        torch.cuda.synchronize()
        f(buf, 1)
        v = dict(zip(NAMES, list(buf)))
        nb = args.blocks
        print(f"== {kind}: per block (cycles), {cb / nb / 1024:.0f} KiB in, {rb / nb / 1024:.0f} KiB out")
        for grp in ("I_", "D_"):
            tot = sum(v[k] for k in NAMES if k.startswith(grp) and k not in COUNTS)
            for k in NAMES:
                if k.startswith(grp):
                    if k in COUNTS:
                        print(f"   {k:10s} {v[k] / nb:14.1f}")
                    else:
                        print(f"   {k:10s} {v[k] / nb:14.0f}  {100 * v[k] / max(tot, 1):5.1f}%")
        del fr, out


if __name__ == "__main__":
    main()
