"""The oracle against frames from an INDEPENDENT encoder (the system liblz4,
tests/golden/make_lz4_fixtures.py): for every ordinary
frame the oracle's output is the encoder's input (digest), which pins the
oracle to liblz4 itself beyond the reference's 24 vectors; for the quirk-D1
frames it is the recorded reference result (lib/lz4ada.adb:811-817, 862-879).
CPU only -- the GPU side is tests/test_gpu_lz4f_fixtures.py."""
import hashlib
import json
import os

import pytest
import xxhash

import _oracle as O
from conftest import GOLDEN

TABLE = json.load(open(os.path.join(GOLDEN, "lz4f_digests.json")))
NAMES = sorted(TABLE["frames"])


def frame(name):
    with open(os.path.join(GOLDEN, "lz4f", name + ".lz4"), "rb") as fh:
        return fh.read()


def test_fixture_set_complete():
    """SURVEY §8c's list: linked 64/256 KiB, independent 64 KiB and 4 MiB, a
    stored/compressed mix, block + content checksum, D1 repros."""
    assert {"linked64k", "linked256k", "indep64k", "indep4m", "mix64k", "d1_cksum"} <= set(NAMES)
    assert sum(n.startswith("d1_") for n in NAMES) >= 4
    assert TABLE["encoder"].startswith("liblz4 1.9")


@pytest.mark.parametrize("name", NAMES)
def test_oracle_on_liblz4_frame(name):
    ent = TABLE["frames"][name]
    data = frame(name)
    assert len(data) == ent["frame_len"]
    st, out, _, msg = O.decode_stream(data)
    assert st == ent["oracle_status"], msg
    if st == O.OK:
        assert {"len": len(out), "sha256": hashlib.sha256(out).hexdigest(),
                "xxh32": xxhash.xxh32(out).intdigest()} == ent["oracle_output"]
    else:
        assert O.exception_information(st, msg) == ent["oracle_error"]
    if not name.startswith("d1_"):
        # the independent encoder's input comes back byte for byte
        assert ent["output_is_input"] and ent["oracle_output"] == ent["input"]


def test_d1_frames_show_the_quirk():
    """At least the shapes whose match reads the literal copy's overshoot
    come back different from the encoder's input (the reference's bytes)."""
    diff = [n for n in NAMES if n.startswith("d1_") and not TABLE["frames"][n]["output_is_input"]]
    assert len(diff) >= 3, diff
