"""The quirk-D1 emulation rule of the linked decoders (lz4ada_idx.hip
d1_emulable, lz4ada_lone.hip k_lone_words), restated in tools/d1_model.py,
against the oracle's bytes (the reference's, D1 corruption included) on the
CPU: every block of a linked frame of 64 KiB generator blocks decoded on top
of the oracle's output before it, with each D1 read emulated -- after
literals (payload bytes) and without literals (the output bytes after the
previous match's source).  No block may differ from the oracle, and both
shapes must occur (lib/lz4ada.adb:790-824, 845-904)."""
import importlib.util
import os

import pytest

import _oracle as O
import lz4ada
import lz4frame

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def model():
    src = open(os.path.join(ROOT, "tools", "d1_model.py")).read().split("nb = int(sys.argv[1])")[0]
    ns = {"__file__": os.path.join(ROOT, "tools", "d1_model.py")}
    exec(compile(src, "d1_model", "exec"), ns)
    return ns


@pytest.mark.parametrize("kind,nb", [("dense", 24), ("mixed", 48)])
def test_d1_rule_matches_oracle(kind, nb):
    m = model()
    blocks = lz4ada.gen_linked_blocks(lz4ada.GEN_KINDS[kind], 0x4C5A3441, 64 << 10, nb)
    frame, _ = lz4frame.build_frame([(c, r, False) for c, r in blocks], 64 << 10, indep=False)
    st, ref, msg = O.unlz4ada(frame, out_cap=nb * (64 << 10) + (1 << 20))
    assert st == O.OK, msg
    reasons, bad = m["emulate"](blocks, ref, True)
    assert bad == [], bad
    assert not any(k.startswith("declined") for k in reasons), reasons
    assert reasons["L>0 k1>0"] > 0
    if kind == "dense":
        assert reasons["L0 k1>0"] > 0
