"""decode_frame wall time (host frame in, host bytes out) for frames of a few
large blocks; run once as is and once with LZ4ADA_NO_LONE=1 to compare the
lone-block path with the bulk decoder."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import lz4ada  # noqa: E402
import lz4frame  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kind", default="mixed")
ap.add_argument("--blocks", default="1,4,16")
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()
for nb in [int(x) for x in args.blocks.split(",")]:
    blocks = [lz4ada.gen_block(lz4ada.GEN_KINDS[args.kind], 77 + i, 4 << 20) + (False,)
              for i in range(nb)]
    frame, raw = lz4frame.build_frame(blocks, 4 << 20, indep=True, block_cksum=True)
    lz4ada.decode_frame(frame)
    ts = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        out, _ = lz4ada.decode_frame(frame)
        ts.append(time.perf_counter() - t0)
    assert out == raw
    ts.sort()
    print(f"{'bulk' if os.environ.get('LZ4ADA_NO_LONE') else 'lone'} {args.kind} {nb} x 4 MiB: "
          f"decode_frame {ts[len(ts) // 2] * 1e3:.2f} ms ({len(raw) / ts[len(ts) // 2] / 2**20:.0f} MiB/s)",
          flush=True)
