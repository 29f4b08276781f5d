#!/usr/bin/env python3
"""Per-phase cycle breakdown of k_decode_blocks (diagnostic build).

    make -C bo-lz4-ada_amd/csrc stamps
    python tools/stamps.py --kind mixed --blocks 512

Loads bo-lz4-ada_amd/liblz4ada_hip_stamps.so (s_memtime stamps between
phases, each stamp drains vmcnt/lgkmcnt, so read SHARES, not totals).
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["LZ4ADA_LIB"] = os.path.join(ROOT, "bo-lz4-ada_amd", "liblz4ada_hip_stamps.so")
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import lz4ada  # noqa: E402
import torch  # noqa: E402

PH = ["stage", "cand", "double", "select", "lit", "match", "flush", "one_token", "wait", "dep"]
CNT = ["batches", "windows", "tokens", "rounds"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="mixed")
    ap.add_argument("--blocks", type=int, default=512)
    ap.add_argument("--unique", type=int, default=16)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    bmax = 4 << 20
    recs = bench.make_unique_blocks(lz4ada.GEN_KINDS[args.kind], args.unique, bmax)
    fr, fl, de, eh, cb, rb, _ = bench.build_shard(recs, 0, args.blocks, bmax, dev)
    out = torch.empty(args.blocks * bmax, dtype=torch.uint8, device=dev)
    st = torch.zeros(args.blocks * 32, dtype=torch.uint8, device=dev)
    f = lz4ada._lib.lz4ada_debug_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 14)()
    lz4ada.launch_decode(fr.data_ptr(), fl, de.data_ptr(), args.blocks, out.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    f(buf, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    lz4ada.launch_decode(fr.data_ptr(), fl, de.data_ptr(), args.blocks, out.data_ptr(), st.data_ptr())
    e1.record()
    torch.cuda.synchronize()
    f(buf, 1)
    v = list(buf)
    tot = sum(v[:10])
    print(f"kind={args.kind} blocks={args.blocks} kernel={e0.elapsed_time(e1):.2f} ms "
          f"(stamped build) decoded={rb / 2**20:.0f} MiB")
    for i, name in enumerate(PH):
        print(f"  {name:10s} {v[i] / args.blocks / 1e6:10.2f} Mcyc/block  {100 * v[i] / max(tot, 1):5.1f}%")
    for i, name in enumerate(CNT):
        print(f"  {name:10s} {v[10 + i] / args.blocks:12.1f} per block")
    nt = max(v[12], 1)
    print(f"  cycles/token {tot / nt:.1f}   tokens/window {v[12] / max(v[11], 1):.2f}   "
          f"tokens/batch {v[12] / max(v[10], 1):.1f}   rounds/batch {v[13] / max(v[10], 1):.2f}")


if __name__ == "__main__":
    main()
