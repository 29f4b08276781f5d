"""Randomised quirk-D1 blocks (lib/lz4ada.adb:790-824,
845-904) through both GPU paths, against the oracle: a full 64 KiB block
(Output_Pos_History = 65,536), an optional small literal block (the D1 block
then starts at Output_Pos n1 > 0), and a crafted block mixing reads 65,529..
65,535 back -- after literals of every length, after no literals, after a
previous match that is in-round, overlapping, from history, or itself a D1
read -- with ordinary in-round and history matches.  Whatever the decoders
emulate or decline, the bytes (bulk: lz4ada_decode_frame) and the call
trace (facade: Update at two feed sizes) must be the reference's.  The
shapes are built here from a seeded PRNG, not from the repo's generator."""
import random
import struct

import pytest

import _oracle as O
import lz4ada
import lz4frame
from test_gpu_facade import trace_oracle, trace_ours_ctx

pytestmark = pytest.mark.gpu
KiB = 1024


def seq(L_bytes, off, ml):
    """One LZ4 sequence: literals, then a match of ml (>= 4) bytes off back."""
    L = len(L_bytes)
    m = ml - 4
    tok = (min(L, 15) << 4) | min(m, 15)
    out = bytes([tok])
    if L >= 15:
        r = L - 15
        while r >= 255:
            out += b"\xff"
            r -= 255
        out += bytes([r])
    out += L_bytes + struct.pack("<H", off)
    if m >= 15:
        r = m - 15
        while r >= 255:
            out += b"\xff"
            r -= 255
        out += bytes([r])
    return out


def lit_only(data):
    """The last sequence of a block: literals only."""
    L = len(data)
    out = bytes([min(L, 15) << 4])
    if L >= 15:
        r = L - 15
        while r >= 255:
            out += b"\xff"
            r -= 255
        out += bytes([r])
    return out + data


def d1_block(rng, n1):
    """A block of 3..14 sequences; positions are output bytes within it."""
    body, pos = b"", 0
    for _ in range(rng.randint(3, 14)):
        L = rng.choice([0, 0, 0, 1, 2, 3, 5, 7, 8, 9, 13, 16, 17, 23, 40])
        lits = bytes(rng.randrange(256) for _ in range(L))
        pos += L
        ml = rng.choice([4, 5, 6, 7, 8, 9, 12, 16, 17, 24, 33, 40])
        shape = rng.random()
        if shape < 0.45:
            # a D1 read: before the round start, within 7 bytes of its end
            off = rng.randint(max(65529, n1 + pos + ml), 65535) if n1 + pos + ml <= 65535 else 0
        elif shape < 0.7 and pos > 0:
            off = rng.randint(1, min(pos, 300))  # in the round (overlapping when off < ml)
        else:
            off = rng.randint(n1 + pos + 1, 65528) if n1 + pos + 1 <= 65528 else 0  # history
        if off == 0:
            off = max(1, pos) if pos > 0 else 65535
        body += seq(lits, off, ml)
        pos += ml
    return body + lit_only(bytes(rng.randrange(256) for _ in range(rng.randint(1, 12))))


@pytest.mark.parametrize("seed", range(120))
def test_d1_fuzz_bulk_and_facade(seed):
    rng = random.Random(0xD1F00 + seed)
    comp0, raw0 = lz4ada.gen_block(1, 1000 + seed, 65536)
    blocks = [(comp0, raw0, False)]
    n1 = rng.choice([0, 0, 0, 1, 7, 40, 300])
    if n1:
        mid = bytes(97 + i % 26 for i in range(n1))
        blocks.append((lit_only(mid), mid, False))
    blocks.append((d1_block(rng, n1), b"", False))
    blocks.append(lz4ada.gen_block(1, 2000 + seed, 30000) + (False,))
    frame, _ = lz4frame.build_frame(blocks, 64 * KiB, indep=False, block_cksum=bool(seed & 1))
    st, ref, msg = O.unlz4ada(frame, out_cap=1 << 20)
    if st == O.OK:
        out, used = lz4ada.decode_frame(frame)
        assert out == ref and used == len(frame)
    else:
        with pytest.raises(lz4ada.LZ4AdaError) as ei:
            lz4ada.decode_frame(frame)
        assert str(ei.value) == O.exception_information(st, msg)
    for feed in (0, 4096):
        ours, _ = trace_ours_ctx(frame, feed)
        assert ours == trace_oracle(frame, feed), feed
