#!/usr/bin/env python3
"""Repeat the literal-class block of tests/test_gpu_multi.py through every
path and report the first wrong byte (diagnostic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import lz4ada  # noqa: E402
import lz4frame  # noqa: E402
from test_gpu_sparse import run_variant  # noqa: E402


def first_diff(a, b):
    n = min(len(a), len(b))
    for i in range(n):
        if a[i] != b[i]:
            return i
    return -1 if len(a) == len(b) else n


def main():
    lens = [4 << 20] * 4
    blocks = [lz4ada.gen_block(i % 4, 3 * 100 + i, n) + (False,) for i, n in enumerate(lens)]
    frame, raw = lz4frame.build_frame(blocks, 4 << 20, indep=True, block_cksum=True)
    c3, r3 = blocks[3][0], blocks[3][1]
    print("block 3: comp", len(c3), "raw", len(r3), "last bytes", r3[-20:].hex())
    for it in range(4):
        out, _ = lz4ada.decode_frame_multi(frame, 1)
        d = first_diff(out, raw)
        print("multi", it, "first diff", d, out[d:d + 20].hex() if d >= 0 else "")
        out, _ = lz4ada.decode_frame(frame)
        d = first_diff(out, raw)
        print("frame", it, "first diff", d)
        info, st, outs = run_variant(frame, lz4ada.DECODE_IDX_SPARSE)
        for b in range(4):
            if st[b].code == 0:
                d = first_diff(outs[b], blocks[b][1])
                if d >= 0:
                    print("  variant block", b, "diff at", d, "len", len(outs[b]), outs[b][d:d + 20].hex(),
                          blocks[b][1][d:d + 20].hex())
            else:
                print("  variant block", b, "code", st[b].code)


if __name__ == "__main__":
    main()
