#!/usr/bin/env python3
"""Time k_decode_wg alone on bench blocks (for rocprofv3 PMC passes).

    python tools/wg_bench.py --kind mixed --blocks 256 --reps 3
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import lz4ada  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kind", default="mixed")
ap.add_argument("--blocks", type=int, default=256)
ap.add_argument("--unique", type=int, default=16)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--wave", action="store_true", help="per-wave decoder instead")
args = ap.parse_args()
dev = torch.device("cuda", 0)
bmax = 4 << 20
recs = bench.make_unique_blocks(lz4ada.GEN_KINDS[args.kind], args.unique, bmax)
fr, fl, de, eh, cb, rb, _ = bench.build_shard(recs, 0, args.blocks, bmax, dev)
out = torch.empty(args.blocks * bmax, dtype=torch.uint8, device=dev)
st = torch.zeros(args.blocks * 32, dtype=torch.uint8, device=dev)
fn = lz4ada.launch_decode if args.wave else lz4ada.launch_decode_wg
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
fn(fr.data_ptr(), fl, de.data_ptr(), args.blocks, out.data_ptr(), st.data_ptr())
torch.cuda.synchronize()
e0.record()
for _ in range(args.reps):
    fn(fr.data_ptr(), fl, de.data_ptr(), args.blocks, out.data_ptr(), st.data_ptr())
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / args.reps
print(f"kind={args.kind} blocks={args.blocks} {'wave' if args.wave else 'wg'} {ms:.3f} ms "
      f"{rb / ms / 1e6:.1f} GB/s out, {(cb + rb) / ms / 1e6:.1f} GB/s alg")
