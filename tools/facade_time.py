#!/usr/bin/env python3
"""Streaming-facade (Init_With_Header + Update loop) throughput on a
synthetic frame, the way tool_unlz4ada drives the library
(unlz4ada.adb:84-103): the input handed over in `--feed`-byte pieces
(0 = all remaining input per call).  Output is checked."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))

import lz4ada  # noqa: E402
import lz4frame  # noqa: E402


def run(frame, expect, feed):
    ctx, used, mbs = lz4ada.Decompressor.init_with_header(frame)
    buf = bytearray(mbs)
    out = bytearray(len(expect) + mbs)  # touched before the timed loop (no page faults in it)
    o = 0
    pos = used
    t0 = time.perf_counter()
    while pos < len(frame):
        stop = len(frame) if feed == 0 else min(len(frame), pos + feed)
        c, f, l = ctx.update(frame, buf, pos, stop)
        if l >= f:
            out[o:o + l + 1 - f] = buf[f:l + 1]
            o += l + 1 - f
        pos += c
        if ctx.is_end_of_frame() == lz4ada.EndOfFrame.Yes:
            break
    dt = time.perf_counter() - t0
    assert bytes(out[:o]) == expect
    return dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="mixed")
    ap.add_argument("--blocks", type=int, default=16)
    ap.add_argument("--block-max", type=int, default=4 << 20)
    ap.add_argument("--feed", type=int, default=0)
    ap.add_argument("--indep", type=int, default=1)
    ap.add_argument("--bcksum", type=int, default=1, help="block checksums in the frame")
    ap.add_argument("--ccksum", type=int, default=1, help="content checksum in the frame")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--raw-len", type=int, default=0,
                    help="decoded bytes per block (default: --block-max)")
    ap.add_argument("--dump", default="",
                    help="also write the frame and its expected output (path, path + '.out') "
                         "for bo-lz4-ada_amd/facade_bench (the same loop from C)")
    args = ap.parse_args()
    n = args.raw_len or args.block_max
    if args.indep:
        blocks = []
        for i in range(args.blocks):
            comp, raw = lz4ada.gen_block(lz4ada.GEN_KINDS[args.kind], 0x4C5A3441 + i, n)
            blocks.append((comp, raw, False))
    else:  # linked: matches reach back into the earlier blocks' output
        blocks = [(c, r, False) for c, r in
                  lz4ada.gen_linked_blocks(lz4ada.GEN_KINDS[args.kind], 0x4C5A3441, n, args.blocks)]
    frame, expect = lz4frame.build_frame(blocks, args.block_max, indep=bool(args.indep),
                                         block_cksum=bool(args.bcksum),
                                          content_cksum=bool(args.ccksum))
    if not args.indep:
        # the reference's bytes (the oracle): with 64 KiB linked blocks quirk
        # D1 can make them differ from the generator's (liblz4's) bytes
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import _oracle as O
        st, ref, msg = O.unlz4ada(frame, out_cap=len(expect) + (1 << 20))
        assert st == O.OK, f"the reference rejects this frame: {msg} (use --ccksum 0)"
        expect = ref
    if args.dump:
        with open(args.dump, "wb") as fh:
            fh.write(frame)
        with open(args.dump + ".out", "wb") as fh:
            fh.write(expect)
    run(frame, expect, args.feed)  # warm
    ts = sorted(run(frame, expect, args.feed) for _ in range(args.reps))
    dt = ts[len(ts) // 2]
    print(f"facade {args.kind} feed={args.feed} bcksum={args.bcksum} ccksum={args.ccksum} "
          f"indep={args.indep} {args.blocks}x{n >> 10} KiB (BD {args.block_max >> 10} KiB) "
          f"decoder={os.environ.get('LZ4ADA_FACADE_DECODER', 'default')}: median of {args.reps} "
          f"{dt * 1e3:.1f} ms  {len(expect) / dt / 2**20:.1f} MiB/s "
          f"(best {len(expect) / ts[0] / 2**20:.1f}, worst {len(expect) / ts[-1] / 2**20:.1f})")


if __name__ == "__main__":
    main()
