"""Errors at the failing block (lz4ada.adb:672-676: the reference checks
block k when it reaches it, after blocks 0..k-1 went out): the bulk path
commits the blocks before the first failing one and the reference-exact
path resumes there, so the partial output and the exception text equal the
oracle's, and a late error costs about one bulk decode, not a redo."""
import random
import time

import pytest

import _oracle as O
import lz4ada
import lz4frame

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not lz4ada.device_available():
        pytest.fail("MI355X not usable: " + lz4ada._thread_error())


def frame_of(sizes, bmax, seed=1, block_cksum=True, content_cksum=True, content_size=False,
             kinds=(1, 0, 3, 2)):
    blocks = []
    for i, n in enumerate(sizes):
        comp, raw = lz4ada.gen_block(kinds[i % len(kinds)], seed * 1000 + i, n)
        blocks.append((comp, raw, False))
    return lz4frame.build_frame(blocks, bmax, indep=True, block_cksum=block_cksum,
                                content_cksum=content_cksum, with_content_size=content_size)


def check_like_oracle(frame):
    st, ref, msg = O.unlz4ada(frame)
    out, cons, exc = lz4ada.decode_frame_partial(frame)
    if st == O.OK:
        assert exc is None and out == ref
    else:
        assert exc is not None and str(exc) == O.exception_information(st, msg)
        assert out == ref  # the blocks the reference output before raising
    return st, exc


def corrupt_payload(frame, k, at=37):
    info, descs = lz4ada.frame_index(frame)
    b = bytearray(frame)
    b[descs[k].in_off + min(at, descs[k].in_len - 1)] ^= 0x5A
    return bytes(b)


@pytest.mark.parametrize("k", [0, 1, 5, 11])
def test_bad_block_checksum_partial_output(k):
    frame, raw = frame_of([65536] * 11 + [4000], 64 << 10)
    st, exc = check_like_oracle(corrupt_payload(frame, k))
    assert isinstance(exc, lz4ada.ChecksumError)
    assert lz4ada.last_path() & lz4ada.PATH_EXACT


@pytest.mark.parametrize("k", [2, 4, 6])
def test_bad_block_after_short_rounds(k):
    # rounds shorter than 64 KiB (lz4ada.adb:678-690): the resume point is
    # the start of the round before the newest one
    sizes = [65536, 65536, 30000, 20000, 65536, 1000, 70000, 500]
    frame, raw = frame_of(sizes, 256 << 10)
    check_like_oracle(corrupt_payload(frame, k))


@pytest.mark.parametrize("seed", range(6))
def test_corrupted_data_without_block_checksum(seed):
    # a flipped byte inside a compressed block: the reference may raise
    # mid-block or decode other bytes; the product answers the same either way
    frame, raw = frame_of([65536] * 8, 64 << 10, seed=seed + 3, block_cksum=False)
    rng = random.Random(seed)
    info, descs = lz4ada.frame_index(frame)
    k = rng.randrange(8)
    b = bytearray(frame)
    b[descs[k].in_off + rng.randrange(descs[k].in_len)] ^= 1 << rng.randrange(8)
    check_like_oracle(bytes(b))


def test_content_checksum_error_outputs_every_block():
    frame, raw = frame_of([65536] * 5, 64 << 10)
    b = bytearray(frame)
    b[-1] ^= 0xFF  # the declared content checksum
    st, exc = check_like_oracle(bytes(b))
    assert isinstance(exc, lz4ada.ChecksumError)


def test_content_size_short_outputs_blocks():
    blocks = [lz4ada.gen_block(1, 90 + i, 65536) for i in range(4)]
    raw = b"".join(r for _, r in blocks)
    hdr = lz4frame.header(64 << 10, indep=True, block_cksum=True, content_size=len(raw) - 1000)
    body = b"".join(lz4frame.block_record(c, block_cksum=True) for c, _ in blocks)
    frame = hdr + body + lz4frame.trailer()
    st, exc = check_like_oracle(frame)
    assert isinstance(exc, lz4ada.DataCorruption)


def test_late_error_in_a_1gib_frame_is_fast():
    """A 1 GiB frame (256 x 4 MiB blocks) whose last block fails its
    checksum raises the oracle's text well under 2 s (the round-2 path redid
    the whole frame first)."""
    bmax = 4 << 20
    uniq = [lz4ada.gen_block(1, 0x4C5A3441 + i, bmax) for i in range(16)]
    blocks = [(uniq[i % 16][0], uniq[i % 16][1], False) for i in range(256)]
    frame, raw = lz4frame.build_frame(blocks, bmax, indep=True, block_cksum=True)
    bad = corrupt_payload(frame, 255, at=1000)
    lz4ada.decode_frame(frame)  # warm (device scratch, code objects)
    t0 = time.perf_counter()
    with pytest.raises(lz4ada.ChecksumError) as ei:
        lz4ada.decode_frame(bad)
    dt = time.perf_counter() - t0
    st, msg = O.error_harness(bad)
    assert str(ei.value) == O.exception_information(st, msg)
    assert dt < 2.0, dt


# ------------------------------------------------ linked frames (D1 included)

def linked_of(lens, bmax, seed, kind=None, content_cksum=True):
    blocks = lz4ada.gen_linked_blocks(kind if kind is not None else lz4ada.GEN_MIXED, seed, 0, 0,
                                      lens=lens)
    frame, raw = lz4frame.build_frame([(c, r, False) for c, r in blocks], bmax, indep=False,
                                      block_cksum=True, content_cksum=content_cksum)
    return frame, blocks


@pytest.mark.parametrize("k", [0, 1, 4, 9])
def test_linked_bad_block_partial_output(k):
    """The linked bulk path resolves the blocks before the bad one and the
    exact path resumes at it over the Buffer they leave (its history)."""
    frame, blocks = linked_of([100000] * 9 + [3000], 256 << 10, seed=40 + k)
    st, exc = check_like_oracle(corrupt_payload(frame, k, at=5000 if k < 9 else 100))
    assert isinstance(exc, lz4ada.ChecksumError)
    if k > 0:
        assert lz4ada.last_path() == lz4ada.PATH_LINKED | lz4ada.PATH_EXACT


@pytest.mark.parametrize("seed", range(4))
def test_linked_corrupted_data_without_block_checksum(seed):
    blocks = lz4ada.gen_linked_blocks(lz4ada.GEN_MIXED, 70 + seed, 0, 0, lens=[65536] * 8)
    frame, raw = lz4frame.build_frame([(c, r, False) for c, r in blocks], 64 << 10, indep=False,
                                      block_cksum=False, content_cksum=True)
    rng = random.Random(seed)
    info, descs = lz4ada.frame_index(frame)
    k = rng.randrange(1, 8)
    b = bytearray(frame)
    b[descs[k].in_off + rng.randrange(descs[k].in_len)] ^= 1 << rng.randrange(8)
    check_like_oracle(bytes(b))


@pytest.mark.parametrize("shape", ["literals", "overlap"])
def test_d1_block_mid_frame(shape):
    """Quirk D1 in block 3 of 5, after blocks 0-2 that
    end at Output_Pos 65536.  'literals': a 20-byte literal run, then the
    read 65533 back -- emulated in the linked bulk path, the whole frame
    there.  'overlap': the read follows a match whose source overlaps its
    output (a repeating part, not emulated) -- blocks 0-2 through the bulk
    path, the exact path from block 3 with the real Buffer."""
    import struct
    pre = lz4ada.gen_linked_blocks(lz4ada.GEN_MIXED, 5, 0, 0, lens=[30000, 20000, 15536])
    if shape == "literals":
        lits = bytes(range(65, 85))
        d1 = bytes([0xF6, 20 - 15]) + lits + struct.pack("<H", 65533) + bytes([0x50]) + b"vwxyz"
    else:
        d1 = (bytes([0x81]) + b"ABCDEFGH" + struct.pack("<H", 3) + bytes([0x06]) +
              struct.pack("<H", 65533) + bytes([0x50]) + b"vwxyz")
    post = lz4ada.gen_block(1, 77, 40000)
    blocks = [(c, r, False) for c, r in pre] + [(d1, b"", False), (post[0], post[1], False)]
    frame, _ = lz4frame.build_frame(blocks, 64 << 10, indep=False, content_cksum=False)
    st, exc = check_like_oracle(frame)
    assert st == O.OK
    want = lz4ada.PATH_LINKED if shape == "literals" else lz4ada.PATH_LINKED | lz4ada.PATH_EXACT
    assert lz4ada.last_path() == want


def test_bulk_resume_checks_declared_content_size():
    """blocks before a failing one that already decode past the
    declared content size -- the reference raises the content-size error in
    the first block that overruns (lz4ada.adb:830-835), not the later
    block's checksum error."""
    blocks = [lz4ada.gen_block(1, 300 + i, 256 << 10) + (False,) for i in range(8)]
    frame, raw = lz4frame.build_frame(blocks, 256 << 10, indep=True, block_cksum=True,
                                      content_cksum=True, with_content_size=True)
    hdr_len = len(lz4frame.header(256 << 10, True, True, True, len(raw)))
    hdr = lz4frame.header(256 << 10, True, True, True, 3 * (256 << 10) + 1000)
    small = bytearray(hdr + frame[hdr_len:])
    info, descs = lz4ada.frame_index(bytes(small))
    small[descs[6].in_off + 40] ^= 0x5A  # block 6's checksum fails
    st, exc = check_like_oracle(bytes(small))
    assert isinstance(exc, lz4ada.DataCorruption) and "content size" in str(exc)
