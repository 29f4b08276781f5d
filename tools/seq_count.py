"""Sequences per launch of a bench class (the denominator of wave
instructions per sequence in DESIGN.md section 4): the bench's unique blocks
(bench.make_unique_blocks) parsed on the host, tiled like the bench frame."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
import lz4ada  # noqa: E402
import lz4frame  # noqa: E402
import xxhash  # noqa: E402


def count(comp):
    p, n, k = 0, len(comp), 0
    while p < n:
        k += 1
        t = comp[p]
        L, x = t >> 4, p + 1
        if L == 15:
            while True:
                e = comp[x]
                x += 1
                L += e
                if e != 255:
                    break
        x += L
        if x >= n:
            break
        x += 2
        if t & 15 == 15:
            while comp[x] == 255:
                x += 1
            x += 1
        p = x
    return k


ap = argparse.ArgumentParser()
ap.add_argument("--kind", default="mixed")
ap.add_argument("--blocks", type=int, default=2048)
ap.add_argument("--unique", type=int, default=64)
args = ap.parse_args()
recs = bench.make_unique_blocks(lz4ada, lz4frame, xxhash, args.kind, args.unique, 4 << 20)
per = [count(r[4]) for r in recs]
total = sum(per[i % len(per)] for i in range(args.blocks))
print(f"{args.kind}: {args.blocks} blocks, {total} sequences ({total / args.blocks:.0f} per block)")
