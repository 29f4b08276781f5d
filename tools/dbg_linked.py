#!/usr/bin/env python3
"""Debug aid (linked bulk path): one linked frame through lz4ada_decode_frame
against the oracle, first differing block; run with LZ4ADA_TRACE_LINKED=3
for per-block statuses and exit reasons.
    python tools/dbg_linked.py KIND BATCH_BYTES [WORDS [CONTENT_CKSUM]]"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))
import importlib.util  # noqa: E402
spec = importlib.util.spec_from_file_location("tl", os.path.join(ROOT, "tests", "test_gpu_linked.py"))
tl = importlib.util.module_from_spec(spec)
spec.loader.exec_module(tl)
import lz4ada  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "mixed"
if len(sys.argv) > 2 and sys.argv[2] != "0":
    os.environ["LZ4ADA_LINKED_BATCH_BYTES"] = sys.argv[2]
if len(sys.argv) > 3 and sys.argv[3] != "auto":
    os.environ["LZ4ADA_LINK_WORDS"] = sys.argv[3]
cck = len(sys.argv) > 4 and sys.argv[4] == "1"
lens = [65536, 70001, 100, 65535, 131075, 3, 65536, 200001, 4097]
frame, raw, blocks = tl.linked_frame(lz4ada.GEN_KINDS[kind], lens, 256 * 1024, seed=17,
                                     content_cksum=cck)
print("model stop", tl.d1_stop(blocks, 256 * 1024), flush=True)
st, ref, msg = tl.oracle(frame)
out, _ = lz4ada.decode_frame(frame)
print("equal", out == ref, "path", lz4ada.last_path(), flush=True)

pos = 0
for k, (c, r) in enumerate(blocks):
    if out[pos:pos + len(r)] != ref[pos:pos + len(r)]:
        a, b = out[pos:pos + len(r)], ref[pos:pos + len(r)]
        j = next(i for i in range(min(len(a), len(b))) if a[i] != b[i]) if len(a) == len(b) else -1
        print(f"block {k} differs at byte {j}: ours {a[j:j+12].hex() if j >= 0 else len(a)} ref {b[j:j+12].hex() if j >= 0 else len(b)}")
        break
    pos += len(r)
