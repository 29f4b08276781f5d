#!/usr/bin/env python3
"""Bulk decode (lz4ada_decode_frame) of a linked frame of 64 KiB blocks
whose uniform offsets put quirk-D1 matches in many blocks: those blocks take
the exact path, and the linked read-ahead batches around them are rebuilt
each time.  Output checked against the oracle (the reference's bytes)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import lz4ada  # noqa: E402
import lz4frame  # noqa: E402
import _oracle as O  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 256
kind = sys.argv[2] if len(sys.argv) > 2 else "mixed"
blocks = lz4ada.gen_linked_blocks(lz4ada.GEN_KINDS[kind], 0x4C5A3441, 64 << 10, nb)
frame, _ = lz4frame.build_frame([(c, r, False) for c, r in blocks], 64 << 10, indep=False)
st, ref, msg = O.unlz4ada(frame, out_cap=nb * (64 << 10) + (1 << 20))
assert st == O.OK, msg
lz4ada.decode_frame(frame)  # warm
ts = []
for _ in range(3):
    t0 = time.perf_counter()
    out, used = lz4ada.decode_frame(frame)
    ts.append(time.perf_counter() - t0)
    assert out == ref
ts.sort()
print(f"d1 frame {kind} {nb} x 64 KiB linked (lib {os.path.basename(lz4ada.LIB_PATH)}): "
      f"median {ts[1] * 1e3:.1f} ms  {len(ref) / ts[1] / 2**20:.1f} MiB/s  path {lz4ada.last_path()}",
      flush=True)
