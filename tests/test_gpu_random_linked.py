"""Randomised LINKED frames through the bulk linked path and the facade,
against the oracle: blocks of ragged sizes whose matches reach up to 65,535
bytes back across block boundaries (the reference decodes every frame as
linked, lib/lz4ada.adb:267-275, 678-690, 845-904), literal runs and matches
of every length class and offsets 1..16, built from a seeded PRNG here (not
the repo's generator).  lz4ada_decode_frame must return the oracle's bytes
(or raise its exception) and Update at 4 KiB feeds must give the oracle's
call trace."""
import random
import struct

import pytest

import _oracle as O
import lz4ada
import lz4frame
from test_gpu_facade import trace_oracle, trace_ours_ctx
from test_gpu_random_blocks import _ext

pytestmark = pytest.mark.gpu


def rand_linked_block(rng, hist, target, exact=False):
    """(payload, decoded) of one block of ~target bytes (exactly target with
    exact=True) after output `hist` (matches may read up to 65,535 bytes
    back, into earlier blocks)."""
    out = bytearray(hist)
    start = len(out)
    comp = bytearray()
    alpha = bytes(rng.choice(range(256)) for _ in range(rng.choice([4, 16, 64])))
    limit = target - 5100 if exact else target
    while len(out) - start < limit:
        r = rng.random()
        L = rng.randint(0, 14) if r < 0.6 else (rng.randint(15, 300) if r < 0.96 else rng.randint(300, 3000))
        if len(out) == 0 and L == 0:
            L = 1
        lits = bytes(rng.choice(alpha) for _ in range(L))
        out += lits
        r = rng.random()
        off = rng.randint(1, 16) if r < 0.3 else (rng.randint(17, 4096) if r < 0.6 else rng.randint(1, 65535))
        if rng.random() < 0.04:
            off = rng.randint(65529, 65535)  # quirk D1's offsets (in a round after a 64 KiB one)
        off = min(off, len(out))
        r = rng.random()
        ml = rng.randint(4, 18) if r < 0.5 else (rng.randint(19, 300) if r < 0.95 else rng.randint(300, 4000))
        m = ml - 4
        comp += bytes([(min(L, 15) << 4) | min(m, 15)])
        if L >= 15:
            comp += _ext(L - 15)
        comp += lits + struct.pack("<H", off)
        if m >= 15:
            comp += _ext(m - 15)
        for _ in range(ml):
            out.append(out[-off])
    n_tail = target - (len(out) - start) if exact else rng.randint(1, 20)
    tail = bytes(rng.choice(alpha) for _ in range(n_tail))
    comp += bytes([min(len(tail), 15) << 4]) + (_ext(len(tail) - 15) if len(tail) >= 15 else b"") + tail
    out += tail
    return bytes(comp), bytes(out[start:])


@pytest.mark.parametrize("seed", range(8))
def test_random_linked_64k_rounds(seed):
    """Every block exactly 64 KiB (LZ4F's default linked frame): each round
    ends at Output_Pos_History = 65,536, so random offsets of 65,529..65,535
    meet quirk D1 after whatever sequence came before -- the reference's
    corrupted bytes (or its content checksum error) from both paths."""
    rng = random.Random(0x64D1 + seed)
    bmax = 64 << 10
    blocks, hist = [], b""
    for _ in range(rng.randint(4, 10)):
        c, r = rand_linked_block(rng, hist[-65536:], bmax, exact=True)
        assert len(r) == bmax
        blocks.append((c, r, False))
        hist += r
    frame, _ = lz4frame.build_frame(blocks, bmax, indep=False, block_cksum=bool(seed & 1))
    st, ref, msg = O.unlz4ada(frame, out_cap=len(hist) + (1 << 20))
    assert st == O.OK, msg
    out, used = lz4ada.decode_frame(frame)
    assert out == ref and used == len(frame)
    for feed in (0, 4096):
        ours, _ = trace_ours_ctx(frame, feed)
        assert ours == trace_oracle(frame, feed), feed


@pytest.mark.parametrize("seed", range(8))
def test_random_linked_frame(seed):
    rng = random.Random(0x11AC + seed)
    bmax = 256 << 10
    blocks, hist = [], b""
    for _ in range(rng.randint(6, 14)):
        target = rng.choice([1, 300, 5000, 40000, 65000, 100000, 200000, 250000])
        c, r = rand_linked_block(rng, hist[-65536:], target)
        assert len(r) <= bmax
        blocks.append((c, r, False))
        hist += r
    frame, _ = lz4frame.build_frame(blocks, bmax, indep=False, block_cksum=bool(seed & 1))
    st, ref, msg = O.unlz4ada(frame, out_cap=len(hist) + (1 << 20))
    if st == O.OK:
        out, used = lz4ada.decode_frame(frame)
        assert out == ref and used == len(frame)
    else:
        with pytest.raises(lz4ada.LZ4AdaError) as ei:
            lz4ada.decode_frame(frame)
        assert str(ei.value) == O.exception_information(st, msg)
    ours, _ = trace_ours_ctx(frame, 4096)
    assert ours == trace_oracle(frame, 4096)
