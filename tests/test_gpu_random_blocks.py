"""Randomised independent blocks through the index decoders, against the
oracle: sequences of every shape the format allows -- literal runs from 0 to
thousands of bytes (length extensions of many 255s), matches 4 bytes to
thousands (RLE-like runs), offsets 1..16 (period patterns), short and up to
64 KiB back -- in ragged block sizes.  Built here from a seeded PRNG, not
from the repo's generator (csrc/lz4gen.cpp), so the decoders' batch cuts,
dealt pieces, ring dependencies and HBM thresholds meet shapes the bench
classes do not have.  Every block a variant accepts must be the oracle's
bytes (lib/lz4ada.adb:716-904); the product path (retry included) must
accept and reproduce every block."""
import random
import struct

import pytest

import lz4ada
import lz4frame
from test_gpu_parity import _run_variant_alone, oracle_blocks

pytestmark = pytest.mark.gpu


def _ext(n):
    out = b""
    while n >= 255:
        out += b"\xff"
        n -= 255
    return out + bytes([n])


def rand_block(rng, target):
    """(payload, decoded) of one block of about `target` decoded bytes."""
    out, comp = bytearray(), bytearray()
    alpha = bytes(rng.randrange(256) for _ in range(rng.choice([4, 16, 64, 256])))
    while len(out) < target:
        r = rng.random()
        L = rng.randint(0, 14) if r < 0.6 else (rng.randint(15, 300) if r < 0.95 else rng.randint(300, 5000))
        if not out and L == 0:
            L = 1
        lits = bytes(rng.choice(alpha) for _ in range(L))
        out += lits
        r = rng.random()
        off = rng.randint(1, 16) if r < 0.35 else (rng.randint(17, 4096) if r < 0.7 else rng.randint(1, 65535))
        off = min(off, len(out))
        r = rng.random()
        ml = rng.randint(4, 18) if r < 0.5 else (rng.randint(19, 300) if r < 0.93 else rng.randint(300, 6000))
        m = ml - 4
        comp += bytes([(min(L, 15) << 4) | min(m, 15)])
        if L >= 15:
            comp += _ext(L - 15)
        comp += lits + struct.pack("<H", off)
        if m >= 15:
            comp += _ext(m - 15)
        for _ in range(ml):
            out.append(out[-off])
    tail = bytes(rng.choice(alpha) for _ in range(rng.randint(1, 20)))
    comp += bytes([min(len(tail), 15) << 4]) + (_ext(len(tail) - 15) if len(tail) >= 15 else b"") + tail
    return bytes(comp), bytes(out + tail)


@pytest.fixture(scope="module")
def frames():
    """Six frames of 20 random blocks each (1 MiB BD, ragged sizes)."""
    res = []
    for seed in range(6):
        rng = random.Random(0xB10C + seed)
        blocks = []
        for _ in range(20):
            target = rng.choice([1, 50, 700, 4095, 16384, 65536, 100000, 250000, 600000])
            c, r = rand_block(rng, target)
            assert len(r) <= 1 << 20
            blocks.append((c, r, False))
        frame, raw = lz4frame.build_frame(blocks, 1 << 20, indep=True, block_cksum=bool(seed & 1))
        res.append((frame, [r for _, r, _ in blocks]))
    return res


@pytest.mark.parametrize("variant", ["product", "idx1", "pp2"])
@pytest.mark.parametrize("k", range(6))
def test_random_blocks(frames, k, variant):
    frame, raws = frames[k]
    ref = oracle_blocks(frame, len(raws))
    assert ref == raws  # the builder's own bytes are the reference's
    v = {"product": lz4ada.DECODE_IDX, "idx1": lz4ada.DECODE_IDX1_ALONE,
         "pp2": lz4ada.DECODE_PP2_ALONE}[variant]
    descs, st, out = _run_variant_alone(frame, v)
    took = 0
    for i, r in enumerate(raws):
        if st[i].code != 0:
            assert variant != "product", (i, st[i].code)
            assert st[i].code in (lz4ada.DS_RETRY, lz4ada.DS_SPARSE), (i, st[i].code)
            continue
        o = descs[i].out_off
        assert st[i].out_len == len(r), i
        assert out[o:o + len(r)] == r, i
        took += 1
    assert took >= len(raws) // 2


@pytest.mark.parametrize("k", range(6))
def test_random_blocks_facade(frames, k):
    """The same frames through Update at 4 KiB feeds (the lone-block decoder
    per block, k_decode_pc below 6 KiB compressed): the oracle's trace."""
    from test_gpu_facade import trace_oracle, trace_ours_ctx
    frame, raws = frames[k]
    ours, exact = trace_ours_ctx(frame, 4096)
    assert ours == trace_oracle(frame, 4096)
