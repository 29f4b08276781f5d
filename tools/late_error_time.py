"""Phase times of a 1 GiB frame (256 x 4 MiB blocks) whose last block fails
its checksum, next to the same frame intact (LZ4ADA_TRACE_FRAME=1 prints
the library's phases to stderr)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "bo-lz4-ada_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import lz4ada  # noqa: E402
import lz4frame  # noqa: E402

bmax = 4 << 20
kind = int(sys.argv[1]) if len(sys.argv) > 1 else 1
uniq = [lz4ada.gen_block(kind, 0x4C5A3441 + i, bmax) for i in range(16)]
blocks = [(uniq[i % 16][0], uniq[i % 16][1], False) for i in range(256)]
frame, raw = lz4frame.build_frame(blocks, bmax, indep=True, block_cksum=True)
info, descs = lz4ada.frame_index(frame)
b = bytearray(frame)
b[descs[255].in_off + 1000] ^= 0x5A
bad = bytes(b)
for rep in range(3):
    t0 = time.perf_counter()
    out, cons = lz4ada.decode_frame(frame)
    t1 = time.perf_counter()
    try:
        lz4ada.decode_frame(bad)
    except lz4ada.ChecksumError:
        pass
    t2 = time.perf_counter()
    print(f"good {1e3 * (t1 - t0):.1f} ms  bad {1e3 * (t2 - t1):.1f} ms", flush=True)
