"""The MI355X path against frames from an independent encoder (the system
liblz4; tests/golden/make_lz4_fixtures.py): each frame
through the streaming facade at 4 KiB reads (tool_unlz4ada's loop,
tool_unlz4ada/unlz4ada.adb:16, 84-103) call by call against the oracle, and
through the bulk path (lz4ada_decode_stream) against the recorded digest."""
import hashlib
import json
import os

import pytest
import xxhash

import _oracle as O
from conftest import GOLDEN
from test_gpu_facade import trace_oracle, trace_ours_ctx

import lz4ada

pytestmark = pytest.mark.gpu

TABLE = json.load(open(os.path.join(GOLDEN, "lz4f_digests.json")))
NAMES = sorted(TABLE["frames"])


def frame(name):
    with open(os.path.join(GOLDEN, "lz4f", name + ".lz4"), "rb") as fh:
        return fh.read()


def digest(b):
    return {"len": len(b), "sha256": hashlib.sha256(b).hexdigest(), "xxh32": xxhash.xxh32(b).intdigest()}


@pytest.mark.parametrize("feed", [4096, 0])
@pytest.mark.parametrize("name", NAMES)
def test_facade_on_liblz4_frame(name, feed):
    data = frame(name)
    ours, exact = trace_ours_ctx(data, feed)
    ref = trace_oracle(data, feed)
    assert len(ours) == len(ref)
    for k, (a, b) in enumerate(zip(ours, ref)):
        assert a == b, f"{name}: call {k}"
    if not name.startswith("d1_"):
        # no block of an ordinary frame needs the reference-exact path
        assert exact == 0, exact


@pytest.mark.parametrize("name", NAMES)
def test_bulk_on_liblz4_frame(name):
    ent = TABLE["frames"][name]
    data = frame(name)
    if ent["oracle_status"] == O.OK:
        out = lz4ada.decode_stream(data)
        assert digest(out) == ent["oracle_output"]
    else:
        with pytest.raises(lz4ada.LZ4AdaError) as ei:
            lz4ada.decode_stream(data)
        assert str(ei.value) == ent["oracle_error"]
