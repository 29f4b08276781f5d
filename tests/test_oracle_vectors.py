"""Pins the CPU oracle to the reference's own fixtures (no GPU).

Mirrors test_suite/lz4test.adb: good vectors at 4 KiB and 1-byte feed
(:250-274), the XXH32 / legacy / raw-block KATs (:129-248), every *.err
vector against its *.eds Exception_Information line (:280-351, :432-447),
and the two hand-written negative cases (:353-430).
"""
import hashlib

import pytest

import _oracle as O
from conftest import error_vectors, good_vectors, read_eds, read_vector


@pytest.mark.parametrize("chunk", [4096, 1], ids=["4K", "1b"])
@pytest.mark.parametrize("name", good_vectors())
def test_good_vector(name, chunk, digests):
    data = read_vector(name, "lz4")
    st, out, eof, msg = O.decode_stream(data, chunk=chunk)
    assert st == O.OK, msg
    assert eof != O.EOF_NO, "Mismatching EOF status"  # lz4test.adb:73-75
    want = digests[name]
    assert len(out) == want["len"]
    assert hashlib.sha256(out).hexdigest() == want["sha256"]
    assert O.xxh32(out) == want["xxh32"]


def test_z9m_reconstruction_matches_declared_checksum():
    # z9m.bin is missing upstream; the frame carries a content checksum, so a
    # successful decode with C.Cksum verified pins the reconstruction.
    data = read_vector("z9m", "lz4")
    assert data[4] & 0x04  # FLG content checksum bit
    st, out, eof, msg = O.decode_stream(data)
    assert st == O.OK, msg
    assert out == bytes(9437166)


def test_xxh32_individual_bytes():
    # lz4test.adb:129-147
    tc = bytes([0x1a] * 14 + [0x11, 0x10])
    h = O.XXH32()
    for b in tc:
        h.update(bytes([b]))
    assert h.final() == 0xf994ef8a
    assert O.xxh32(tc) == 0xf994ef8a


def test_xxh32_init_ignores_seed():
    # Quirk Q1: XXHash32.Init(Seed) ignores Seed (lz4ada.adb:925-930);
    # Reset(Seed) honours it (lz4ada.adb:932-940).
    a = O.XXH32(seed=1234)
    a.update(b"abc")
    assert a.final() == O.xxh32(b"abc")
    a.reset(1234)
    a.update(b"abc")
    import xxhash
    assert a.final() == xxhash.xxh32(b"abc", seed=1234).intdigest()


def test_xxh32_against_python_xxhash():
    import random
    import xxhash
    rng = random.Random(7)
    for n in [0, 1, 3, 4, 15, 16, 17, 31, 32, 33, 100, 1000, 4097]:
        data = bytes(rng.getrandbits(8) for _ in range(n))
        assert O.xxh32(data) == xxhash.xxh32(data).intdigest()
        h = O.XXH32()
        i = 0
        while i < n:  # ragged update sizes
            k = rng.randint(1, 40)
            h.update(data[i:i + k])
            i += k
        assert h.final() == xxhash.xxh32(data).intdigest()


LEGACY_TC = bytes.fromhex(
    "02214c1830000000f01f3c3f786d6c2076657273696f6e3d22312e302220656e636f"
    "64696e673d225554462d38223f3e3c746573742f3e0a02214c180e000000d048656c"
    "6c6f20776f726c642e0a")


def test_decompress_individual_bytes():
    # lz4test.adb:149-214: Init_With_Header(For_All) then 1-byte Updates.
    expect = b'<?xml version="1.0" encoding="UTF-8"?><test/>\nHello world.\n'
    st, msg, ctx, consumed = O.Decompressor.init_with_header(LEGACY_TC, O.FOR_ALL)
    assert st == O.OK, msg
    import ctypes
    buf = ctypes.create_string_buffer(ctx.min_buffer_size)
    have = b""
    for i in range(consumed, len(LEGACY_TC)):
        nc = 0
        while nc == 0:
            st, nc, f, l = ctx.update(LEGACY_TC[i:i + 1], buf)
            assert st == O.OK, ctx.last_error()
            assert not (nc == 0 and l < f), "no output produced but expected"
            if l >= f:
                have += buf.raw[f:l + 1]
    assert have == expect


def test_hello_block():
    # lz4test.adb:216-248: Init_For_Block + one Update.
    import ctypes
    tc = bytes.fromhex("d048656c6c6f2c20776f726c642e")
    ctx = O.Decompressor.init_for_block(len(tc))
    buf = ctypes.create_string_buffer(ctx.min_buffer_size)
    st, nc, f, l = ctx.update(tc, buf)
    assert st == O.OK
    assert nc == len(tc)
    assert ctx.is_end_of_frame() == O.EOF_YES
    assert buf.raw[:13] == b"Hello, world."
    assert (f, l) == (0, 12)


@pytest.mark.parametrize("name", error_vectors())
def test_error_vector(name):
    # lz4test.adb:280-351: whole .err file (<= 10,001 bytes, :328) through
    # Init_With_Header(Single_Frame) + Update; the raised exception's
    # information must equal the .eds line exactly.
    data = read_vector(name, "err")[:10001]
    st, msg = O.error_harness(data)
    assert st in (O.CHECKSUM_ERROR, O.DATA_CORRUPTION, O.NOT_SUPPORTED,
                  O.TOO_FEW_HEADER_BYTES, O.TOO_LITTLE_MEMORY), (st, msg)
    assert O.exception_information(st, msg) == read_eds(name)


def test_reservation_exceeded():
    # lz4test.adb:353-382: first 36 bytes of z2841 (BD = 1 MiB) with SZ_64_KiB.
    tc = read_vector("z2841", "lz4")[:36]
    st, msg, ctx, _ = O.Decompressor.init_with_header(tc, O.SZ_64_KIB)
    assert st == O.TOO_LITTLE_MEMORY
    assert msg.startswith("LZ4 header requres reservation SZ_1_MIB, but API call "
                          "requested that only SZ_64_KIB be used.")


def test_unexpected_multi_frame():
    # lz4test.adb:384-430: two minilegacy frames under Single_Frame.
    import ctypes
    tc = read_vector("minilegacy", "lz4") * 2
    st, msg, ctx, total = O.Decompressor.init_with_header(tc, O.SINGLE_FRAME)
    assert st == O.OK
    buf = ctypes.create_string_buffer(ctx.min_buffer_size)
    while total < len(tc):
        st, nc, f, l = ctx.update(tc[total:], buf)
        if st:
            break
        total += nc
    assert st == O.DATA_CORRUPTION


def test_unlz4ada_cli_config1(digests):
    # Config C1: z100.lz4 through the unlz4ada loop (tool_unlz4ada.adb:63-105).
    st, out, msg = O.unlz4ada(read_vector("z100", "lz4"))
    assert st == O.OK, msg
    assert hashlib.sha256(out).hexdigest() == digests["z100"]["sha256"]
    assert digests["z100"]["sha256"].startswith("cd00e292c5970d3c")


@pytest.mark.parametrize("name", ["z1", "t2", "t389", "t100k", "t300k", "t1111k", "z2841",
                                  "concat390", "skipz100"])
def test_unlz4ada_cli_modern(name, digests):
    st, out, msg = O.unlz4ada(read_vector(name, "lz4"))
    assert st == O.OK, msg
    assert hashlib.sha256(out).hexdigest() == digests[name]["sha256"]
