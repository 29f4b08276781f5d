"""GPU parity tests: the MI355X decoder (through its C-ABI) against the
reference's fixtures and the CPU oracle.  Mirrors test_suite/lz4test.adb.
"""
import hashlib
import random

import pytest

import _oracle as O
from conftest import error_vectors, good_vectors, read_eds, read_vector

import lz4ada
import lz4frame

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not lz4ada.device_available():
        pytest.fail("MI355X not usable: " + lz4ada._thread_error())


def feed(ctx, mbs, data, chunk):
    """lz4test.adb:32-83 (Test_Good_Case_Inner) over the product."""
    buf = bytearray(mbs)
    out = bytearray()
    pos = 0
    eof = ctx.is_end_of_frame()
    while pos < len(data):
        win_end = min(pos + chunk, len(data))
        used = pos
        while used < win_end:
            c, f, l = ctx.update(data, buf, used, win_end)
            if l >= f:
                out += buf[f:l + 1]
            used += c
            eof = ctx.is_end_of_frame()
        pos = win_end
    return bytes(out), eof


def feed_bytes(ctx, mbs, data):
    """feed() with chunk 1 (lz4test.adb:252), one byte per Update call, with
    the ctypes call bound once so that multi-MB vectors stay in seconds."""
    import ctypes
    buf = bytearray(mbs)
    cbuf = (ctypes.c_char * max(mbs, 1)).from_buffer(buf)
    out = bytearray()
    upd = lz4ada._lib.lz4ada_update
    cons, first, last = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    rc, rf, rl = ctypes.byref(cons), ctypes.byref(first), ctypes.byref(last)
    src = ctypes.create_string_buffer(bytes(data), len(data))
    base = ctypes.addressof(src)
    p = ctx._p
    for i in range(len(data)):
        used = 0
        while used < 1:
            st = upd(p, base + i + used, 1 - used, rc, cbuf, mbs, rf, rl)
            if st:
                lz4ada._check(st, lz4ada._lib.lz4ada_last_error(p).decode())
            if last.value >= first.value:
                out += buf[first.value:last.value + 1]
            used += cons.value
    return bytes(out), ctx.is_end_of_frame()


def check_digest(out, want):
    assert len(out) == want["len"]
    assert hashlib.sha256(out).hexdigest() == want["sha256"]


@pytest.mark.parametrize("chunk", [4096, 1], ids=["4K", "1b"])
@pytest.mark.parametrize("name", good_vectors())
def test_good_vector_streaming(name, chunk, digests):
    data = read_vector(name, "lz4")
    ctx, mbs = lz4ada.Decompressor.init(lz4ada.FOR_ALL)
    out, eof = feed(ctx, mbs, data, chunk) if chunk > 1 else feed_bytes(ctx, mbs, data)
    assert eof != lz4ada.EndOfFrame.No
    check_digest(out, digests[name])


@pytest.mark.parametrize("name", good_vectors())
def test_good_vector_bulk(name, digests):
    data = read_vector(name, "lz4")
    out = lz4ada.decode_stream(data)
    check_digest(out, digests[name])


def test_xxh32_individual_bytes():
    tc = bytes([0x1a] * 14 + [0x11, 0x10])
    h = lz4ada.XXHash32()
    for b in tc:
        h.update(bytes([b]))
    assert h.final() == 0xf994ef8a
    assert lz4ada.XXHash32.hash(tc) == 0xf994ef8a


def test_xxh32_random_against_oracle():
    rng = random.Random(3)
    for n in [0, 1, 15, 16, 17, 255, 256, 1023, 1024, 1025, 4096 + 3, 100_000, 1 << 20]:
        data = rng.randbytes(n + 7)
        for off in (0, 1, 3):
            chunk = data[off:off + n]
            assert lz4ada.XXHash32.hash(chunk) == O.xxh32(chunk), (n, off)
    h = lz4ada.XXHash32()
    data = rng.randbytes(50_000)
    i = 0
    while i < len(data):
        k = rng.randint(1, 3000)
        h.update(data[i:i + k])
        i += k
    assert h.final() == O.xxh32(data)


@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 1000, (32 << 20) - 3, (32 << 20) + 16 + 5,
                               (64 << 20) + 9])
def test_content_checksum_pipeline(n):
    """lz4ada_content_xxh32_d2h (D2H + host chain) equals the oracle's XXH32
    and delivers the bytes; its state continues the GPU chain's and back."""
    import torch
    g = torch.Generator().manual_seed(n)
    host = torch.randint(0, 256, (n + 64,), dtype=torch.uint8, generator=g)
    d = host.cuda()
    data = bytes(host[:n].numpy())
    want = O.xxh32(data)
    h = lz4ada.XXHash32()
    out = bytearray(n)
    h.update_device_d2h(d.data_ptr(), n, out)
    assert h.final() == want
    assert bytes(out) == data
    # split: GPU chain for an odd prefix, host pipeline for the rest, and back
    k = n // 3 + 1 if n else 0
    h = lz4ada.XXHash32()
    h.update_device(d.data_ptr(), k)
    h.update_device_d2h(d.data_ptr() + k, max(n - k - 5, 0))
    h.update_device(d.data_ptr() + k + max(n - k - 5, 0), n - k - max(n - k - 5, 0))
    assert h.final() == want


def test_decompress_individual_bytes():
    # lz4test.adb:149-214
    tc = bytes.fromhex(
        "02214c1830000000f01f3c3f786d6c2076657273696f6e3d22312e302220656e636f"
        "64696e673d225554462d38223f3e3c746573742f3e0a02214c180e000000d048656c"
        "6c6f20776f726c642e0a")
    expect = b'<?xml version="1.0" encoding="UTF-8"?><test/>\nHello world.\n'
    ctx, consumed, mbs = lz4ada.Decompressor.init_with_header(tc, lz4ada.FOR_ALL)
    buf = bytearray(mbs)
    have = b""
    for i in range(consumed, len(tc)):
        nc = 0
        while nc == 0:
            nc, f, l = ctx.update(tc, buf, i, i + 1)
            assert not (nc == 0 and l < f)
            if l >= f:
                have += bytes(buf[f:l + 1])
    assert have == expect


def test_hello_block():
    # lz4test.adb:216-248
    tc = bytes.fromhex("d048656c6c6f2c20776f726c642e")
    ctx, mbs = lz4ada.Decompressor.init_for_block(len(tc))
    buf = bytearray(mbs)
    c, f, l = ctx.update(tc, buf)
    assert c == len(tc)
    assert ctx.is_end_of_frame() == lz4ada.EndOfFrame.Yes
    assert bytes(buf[:13]) == b"Hello, world."


def error_harness(data):
    """lz4test.adb:280-308 over the product."""
    ctx, total, mbs = lz4ada.Decompressor.init_with_header(data, lz4ada.Reservation.Single_Frame)
    buf = bytearray(mbs)
    while total < len(data):
        c, f, l = ctx.update(data, buf, total)
        assert c != 0, "No more data accepted but no exception signalled"
        total += c
    raise AssertionError("All data processed but no exception raised")


@pytest.mark.parametrize("name", error_vectors())
def test_error_vector(name):
    data = read_vector(name, "err")[:10001]
    with pytest.raises(lz4ada.LZ4AdaError) as ei:
        error_harness(data)
    assert str(ei.value) == read_eds(name)


def test_unexpected_multi_frame():
    tc = read_vector("minilegacy", "lz4") * 2
    with pytest.raises(lz4ada.DataCorruption):
        error_harness(tc)


# ------------------------------------------------ synthetic frames (bulk)

def synth_frame(kind, nblocks, block_max, seed=0, last_short=True, block_cksum=True,
                content_cksum=True, indep=True, stored_every=0):
    blocks = []
    for i in range(nblocks):
        raw_len = block_max
        if last_short and i == nblocks - 1:
            raw_len = block_max // 3 + 17
        if stored_every and i % stored_every == stored_every - 1:
            raw = random.Random(seed + i).randbytes(raw_len)
            blocks.append((raw, raw, True))
        else:
            comp, raw = lz4ada.gen_block(kind, seed * 1000 + i, raw_len)
            blocks.append((comp, raw, False))
    return lz4frame.build_frame(blocks, block_max, indep=indep, block_cksum=block_cksum,
                                content_cksum=content_cksum)


@pytest.mark.parametrize("kind", ["dense", "mixed", "rle", "literal"])
@pytest.mark.parametrize("block_max", [64 << 10, 4 << 20])
def test_synthetic_independent_frame(kind, block_max):
    nb = 6 if block_max == 64 << 10 else 3
    frame, raw = synth_frame(lz4ada.GEN_KINDS[kind], nb, block_max, seed=5, stored_every=4)
    out, consumed = lz4ada.decode_frame(frame)
    assert consumed == len(frame)
    assert out == raw
    st, oref, eof, msg = O.decode_stream(frame)
    assert st == O.OK and oref == raw


def test_synthetic_short_middle_blocks_compact():
    # non-last blocks shorter than block_max force the compaction pass
    blocks = []
    for i, n in enumerate([1000, 65536, 5, 40000, 65536, 777]):
        comp, raw = lz4ada.gen_block(i % 4, 77 + i, n)
        blocks.append((comp, raw, False))
    frame, raw = lz4frame.build_frame(blocks, 64 << 10, block_cksum=True, content_cksum=True)
    out, _ = lz4ada.decode_frame(frame)
    assert out == raw


def test_bulk_errors_fall_back_to_exact_messages():
    frame, raw = synth_frame(0, 4, 64 << 10, seed=9)
    # flip a byte inside block 2's payload -> its block checksum fails
    info, descs = lz4ada.frame_index(frame)
    bad = bytearray(frame)
    bad[descs[2].in_off + 100] ^= 0x55
    with pytest.raises(lz4ada.ChecksumError) as ei:
        lz4ada.decode_frame(bytes(bad))
    st, msg = O.error_harness(bytes(bad))
    assert str(ei.value) == O.exception_information(st, msg)


def test_device_resident_blocks():
    torch = pytest.importorskip("torch")
    import ctypes
    frame, raw = synth_frame(1, 8, 64 << 10, seed=11, stored_every=3)
    info, descs = lz4ada.frame_index(frame)
    nb = info.nblocks
    dev = torch.device("cuda:0")
    d_frame = torch.frombuffer(bytearray(frame), dtype=torch.uint8).to(dev)
    d_desc = torch.frombuffer(bytearray(bytes(descs)[:nb * 32]), dtype=torch.uint8).to(dev)
    d_out = torch.zeros(nb * info.block_max, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(nb * 32, dtype=torch.uint8, device=dev)
    d_hash = torch.zeros(nb, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    lz4ada.decode_blocks_device(d_frame.data_ptr(), len(frame), d_desc.data_ptr(), nb,
                                d_out.data_ptr(), d_st.data_ptr(), stream)
    torch.cuda.synchronize()
    st = (lz4ada.BlockStatus * nb).from_buffer_copy(d_st.cpu().numpy().tobytes())
    total = sum(s.out_len for s in st)
    assert total == len(raw)
    assert all(s.code == 0 for s in st)
    for i in range(nb):
        if descs[i].flags & lz4ada.BLOCK_HAS_CKSUM:
            assert st[i].cksum == descs[i].cksum
    assert bytes(d_out.cpu().numpy()[:total]) == raw


# ------------------------------------------- bench-sized blocks (regression)

@pytest.mark.parametrize("variant", ["pc", "idx", "idx1"])
@pytest.mark.parametrize("kind", ["dense", "mixed", "rle", "literal"])
def test_bench_blocks_exact(kind, variant):
    """The bench's own unique 4 MiB blocks (seed 0x4C5A3441 + i) decode
    byte-exactly through every bulk decoder."""
    torch = pytest.importorskip("torch")
    seeds = [0x4C5A3441 + i for i in range(16)]
    bmax = 4 << 20
    blocks = [lz4ada.gen_block(lz4ada.GEN_KINDS[kind], sd, bmax) for sd in seeds]
    frame, raw = lz4frame.build_frame([(c, r, False) for c, r in blocks], bmax,
                                      block_cksum=True)
    info, descs = lz4ada.frame_index(frame)
    nb = info.nblocks
    dev = torch.device("cuda:0")
    d_frame = torch.frombuffer(bytearray(frame), dtype=torch.uint8).to(dev)
    d_desc = torch.frombuffer(bytearray(bytes(descs)[:nb * 32]), dtype=torch.uint8).to(dev)
    d_out = torch.zeros(nb * bmax, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(nb * 32, dtype=torch.uint8, device=dev)
    sh = torch.cuda.current_stream().cuda_stream
    lz4ada.launch_block_checksums(d_frame.data_ptr(), d_desc.data_ptr(), nb, d_st.data_ptr(), sh)
    v = {"pc": lz4ada.DECODE_PC, "idx": lz4ada.DECODE_IDX,
         "idx1": lz4ada.DECODE_IDX1_ALONE}[variant]
    lz4ada.launch_decode_variant(d_frame.data_ptr(), len(frame), d_desc.data_ptr(), nb,
                                 d_out.data_ptr(), d_st.data_ptr(), v, sh)
    torch.cuda.synchronize()
    st = (lz4ada.BlockStatus * nb).from_buffer_copy(d_st.cpu().numpy().tobytes())
    out = d_out.cpu().numpy().tobytes()
    bad = []
    for i, (c, r) in enumerate(blocks):
        assert st[i].cksum == descs[i].cksum, (i, "block checksum")
        if variant == "idx1" and st[i].code == lz4ada.DS_SPARSE:
            continue  # the index decoder alone leaves these to k_decode_sparse
        got = out[i * bmax:i * bmax + len(r)]
        if st[i].code or st[i].out_len != len(r) or got != r:
            j = next((k for k in range(len(r)) if got[k] != r[k]), -1)
            bad.append((i, st[i].code, st[i].out_len, j,
                        got[max(j - 8, 0):j + 8].hex(), r[max(j - 8, 0):j + 8].hex()))
    assert not bad, bad


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 3])
def test_sharded_decode_each_rank_share(world):
    """shard.decode_frame_sharded for every rank of a world (no process group:
    the status reduce is local), reassembled against the oracle."""
    import shard
    import torch
    blocks = []
    for i in range(7):
        raw_len = 256 * 1024 if i < 6 else 1000
        comp, raw = lz4ada.gen_block(i % 4, 0x4C5A3441 + i, raw_len)
        blocks.append((comp, raw, False))
    frame, expected = lz4frame.build_frame(blocks, 256 * 1024, indep=True, block_cksum=True)
    got = b""
    for rank in range(world):
        d_out, (lo, hi), lens = shard.decode_frame_sharded(frame, rank, world,
                                                          torch.device("cuda", 0))
        host = d_out.cpu().numpy().tobytes()
        for j, ln in enumerate(lens):
            got += host[j * 256 * 1024:j * 256 * 1024 + ln]
    assert got == expected


def _run_variant_alone(frame, variant):
    """Decode a frame's blocks with one decoder variant and no retry pass;
    returns (descs, statuses, output bytes)."""
    import torch
    info, descs = lz4ada.frame_index(frame)
    nb = info.nblocks
    bmax = info.block_max
    dev = torch.device("cuda:0")
    d_frame = torch.frombuffer(bytearray(frame), dtype=torch.uint8).to(dev)
    d_desc = torch.frombuffer(bytearray(bytes(descs)[:nb * 32]), dtype=torch.uint8).to(dev)
    d_out = torch.zeros(nb * bmax, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(nb * 32, dtype=torch.uint8, device=dev)
    lz4ada.launch_decode_variant(d_frame.data_ptr(), len(frame), d_desc.data_ptr(), nb,
                                 d_out.data_ptr(), d_st.data_ptr(), variant,
                                 torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    st = (lz4ada.BlockStatus * nb).from_buffer_copy(d_st.cpu().numpy().tobytes())
    return descs, st, d_out.cpu().numpy().tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["default", "idx1", "pp2"])
@pytest.mark.parametrize("kind", ["dense", "mixed", "literal", "rle", "chain"])
@pytest.mark.parametrize("bmax", [64 << 10, 256 << 10, 4 << 20])
def test_idx_decoder_alone(kind, bmax, variant):
    """k_index + k_decode_idx on their own: exact output for every block they
    accept, and they accept every well-formed independent block except sparse
    large ones (long literal runs: over 64 input bytes per sequence), which
    they leave (status DS_SPARSE) to the literal-heavy decoder, and RLE blocks of
    at least 4 KiB input with over 64 output bytes (slot) per input byte."""
    blocks = [lz4ada.gen_block(lz4ada.GEN_KINDS[kind], 0x4C5A3441 + i, bmax) for i in range(6)]
    blocks.append(lz4ada.gen_block(lz4ada.GEN_KINDS[kind], 77, 1000))  # short last block
    # ragged sizes: partial pass-1 chunks and batches, both waves' shares
    for j, n in enumerate((bmax - 1, bmax // 2 + 33, 16384 + 5, 4097, 200, 17, 1)):
        blocks.append(lz4ada.gen_block(lz4ada.GEN_KINDS[kind], 900 + j, min(n, bmax)))
    frame, raw = lz4frame.build_frame([(c, r, False) for c, r in blocks], bmax, indep=True)
    v = {"default": lz4ada.DECODE_IDX_ALONE, "idx1": lz4ada.DECODE_IDX1_ALONE,
         "pp2": lz4ada.DECODE_PP2_ALONE}[variant]
    descs, st, out = _run_variant_alone(frame, v)
    bad = []
    for i, (c, r) in enumerate(blocks):
        if kind == "literal" and st[i].code == lz4ada.DS_SPARSE and len(c) >= 65536:
            continue
        if st[i].code == lz4ada.DS_SPARSE and len(c) >= 4096 and len(c) * 64 < bmax:
            continue  # over 64 slot bytes per input byte: the scalar-parse decoder's
        got = out[i * bmax:i * bmax + len(r)]
        if st[i].code or st[i].out_len != len(r) or got != r:
            j = next((k for k in range(min(len(r), len(got))) if got[k] != r[k]), -1)
            bad.append((i, st[i].code, st[i].out_len, len(r), j))
    assert not bad, bad


@pytest.mark.gpu
def test_idx_decoder_stored_and_small():
    """Stored blocks, tiny blocks and an empty block through the idx decoder."""
    blocks = []
    for i in range(9):
        raw_len = [65536, 1, 0, 13, 100, 65536, 4000, 31, 33][i]
        if i in (5, 6):
            raw = random.Random(500 + i).randbytes(raw_len)
            blocks.append((raw, raw, True))
        else:
            comp, raw = lz4ada.gen_block(i % 4, 500 + i, raw_len)
            blocks.append((comp, raw, False))
    frame, raw = lz4frame.build_frame(blocks, 64 << 10, indep=True, block_cksum=True)
    info, descs = lz4ada.frame_index(frame)
    descs_, st, out = _run_variant_alone(frame, lz4ada.DECODE_IDX)
    got = b"".join(out[i * info.block_max:i * info.block_max + st[i].out_len]
                   for i in range(info.nblocks))
    assert all(s.code == 0 for s in st[:info.nblocks])
    assert got == raw


def oracle_blocks(frame, nblocks):
    """The first frame's blocks as the oracle's Update returns them (one per
    call; zero-length blocks included, from the size words)."""
    import ctypes
    info, descs = lz4ada.frame_index(frame)
    ctx = O.Decompressor.init()
    buf = ctypes.create_string_buffer(ctx.min_buffer_size)
    blocks, pos = [], 0
    while len(blocks) < nblocks and pos < len(frame):
        st, c, f, l = ctx.update(frame[pos:pos + 4096], buf)
        assert st == O.OK, ctx.last_error()
        if l >= f:
            blocks.append(buf.raw[f:l + 1])
        pos += c
        # a block that decodes to nothing returns no output: account for it
        while len(blocks) < nblocks and descs[len(blocks)].in_len == 0 and \
                not descs[len(blocks)].flags & lz4ada.BLOCK_STORED:
            blocks.append(b"")
    return blocks


@pytest.mark.gpu
@pytest.mark.parametrize("alone", ["default", "idx1", "pp2"])
@pytest.mark.parametrize("name", ["t100k", "t1111k", "b3444k", "z2841", "t300k", "a2246", "z9m"])
def test_idx_decoder_on_vectors(name, digests, alone):
    """Reference vectors' blocks through the idx decoder (+ retry): every block
    byte-exact; linked blocks that reference earlier blocks are declined
    (DS_RETRY) by the idx pass and redone exactly."""
    frame = read_vector(name, "lz4")
    info, _ = lz4ada.frame_index(frame)
    v = {"default": lz4ada.DECODE_IDX_ALONE, "idx1": lz4ada.DECODE_IDX1_ALONE,
         "pp2": lz4ada.DECODE_PP2_ALONE}[alone]
    descs, st, out = _run_variant_alone(frame, v)
    for i in range(info.nblocks):
        assert st[i].code in (0, lz4ada.DS_RETRY, lz4ada.DS_SPARSE), (i, st[i].code)
    ref = oracle_blocks(frame, info.nblocks)
    for i in range(info.nblocks):  # every block the index decoder alone took
        if st[i].code == 0:
            assert out[i * info.block_max:i * info.block_max + st[i].out_len] == ref[i], i
    descs, st, out = _run_variant_alone(frame, lz4ada.DECODE_IDX)
    pieces = [out[i * info.block_max:i * info.block_max + st[i].out_len]
              for i in range(info.nblocks)]
    if all(s.code == 0 for s in st[:info.nblocks]):
        assert hashlib.sha256(b"".join(pieces)).hexdigest() == digests[name]["sha256"]
    # block by block against the oracle's Update outputs (one block per
    # call, lz4ada.adb:383-418), for every block the bulk decoders took --
    # also when others were declined
    ref = oracle_blocks(frame, info.nblocks)
    assert len(ref) == info.nblocks
    took = [i for i in range(info.nblocks) if st[i].code == 0]
    assert took or not info.nblocks, "no block was decoded"
    for i in took:
        assert pieces[i] == ref[i], i


# ------------------------------------------- linked frames (BASELINE configs[4])

@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["dense", "mixed", "rle", "literal"])
def test_linked_frame_fast_path(kind):
    """A linked 256 KiB-block frame whose matches reach into the previous
    block (configs[4] shape, small): the in-order index-driven path decodes
    every block itself (no decline) and byte-exactly; decode_frame agrees
    with the oracle."""
    blocks = lz4ada.gen_linked_blocks(lz4ada.GEN_KINDS[kind], 0x4C5A3441, 256 << 10, 6,
                                      last_len=70000)
    frame, raw = lz4frame.build_frame([(c, r, False) for c, r in blocks], 256 << 10,
                                      indep=False, block_cksum=True, content_cksum=True)
    st_o, ref, _, msg = O.decode_stream(frame)
    assert st_o == O.OK and ref == raw, msg
    descs, st, out = _run_variant_alone(frame, lz4ada.DECODE_IDX_LINKED)
    info, _ = lz4ada.frame_index(frame)
    assert not info.independent
    if kind != "literal":  # sparse literal blocks are declined (exact path)
        assert all(s.code == 0 for s in st[:info.nblocks]), [s.code for s in st[:info.nblocks]]
    if all(s.code == 0 for s in st[:info.nblocks]):
        got = b"".join(out[i * info.block_max:i * info.block_max + st[i].out_len]
                       for i in range(info.nblocks))
        assert got == raw
    dec, consumed = lz4ada.decode_frame(frame)
    assert consumed == len(frame) and dec == raw


@pytest.mark.gpu
def test_linked_frame_short_block_falls_back():
    """A short middle block breaks the slot layout: the linked path leaves
    the rest to the exact path, and the frame still decodes exactly."""
    blocks = lz4ada.gen_linked_blocks(1, 7, 256 << 10, 3)
    c, r = lz4ada.gen_linked_blocks(1, 8, 5000, 1)[0]  # no history: valid anywhere
    blocks.insert(1, (c, r))
    frame, raw = lz4frame.build_frame([(c, r, False) for c, r in blocks], 256 << 10,
                                      indep=False, block_cksum=True)
    descs, st, out = _run_variant_alone(frame, lz4ada.DECODE_IDX_LINKED)
    assert st[0].code == 0 and st[1].code == 0
    assert all(s.code == lz4ada.DS_RETRY for s in st[2:4])
    # (the blocks after the inserted one were generated against other
    # history, so the oracle, not `raw`, says what the frame decodes to)
    st_o, ref, _, msg = O.decode_stream(frame)
    assert st_o == O.OK, msg
    dec, consumed = lz4ada.decode_frame(frame)
    assert dec == ref


@pytest.mark.gpu
def test_linked_frame_64k():
    """64 KiB linked blocks (the LZ4F default): the bulk linked path, or the
    exact path where the reference's D1 overshoot could matter; output
    equals the oracle's either way (tests/test_gpu_linked.py checks which)."""
    blocks = lz4ada.gen_linked_blocks(1, 11, 64 << 10, 4)
    frame, raw = lz4frame.build_frame([(c, r, False) for c, r in blocks], 64 << 10,
                                      indep=False)
    st_o, ref, _, msg = O.decode_stream(frame)
    assert st_o == O.OK, msg
    dec, consumed = lz4ada.decode_frame(frame)
    assert dec == ref


@pytest.mark.parametrize("nblocks", [40, 1100])  # two-wave (<= 4 x CUs) and one-wave fused decoder
def test_stored_blocks_hashed_while_copied(nblocks):
    """Stored blocks with B.Checksum through the fused decoders (two-wave
    and one-wave): copied by the decoder, hashed beside it -- every size
    class of the 16-byte stripe loop and its tail, every payload alignment,
    against the frame's declared checksums and the oracle."""
    torch = pytest.importorskip("torch")
    sizes = [1, 15, 16, 17, 255, 1000, 8191, 8192, 8193, 20000, 65536]
    blocks = []
    for i in range(nblocks):
        raw = random.Random(900 + i).randbytes(sizes[i % len(sizes)])
        blocks.append((raw, raw, True))
    frame, raw = lz4frame.build_frame(blocks, 64 << 10, block_cksum=True)
    info, descs = lz4ada.frame_index(frame)
    nb = info.nblocks
    dev = torch.device("cuda:0")
    d_frame = torch.frombuffer(bytearray(frame), dtype=torch.uint8).to(dev)
    d_desc = torch.frombuffer(bytearray(bytes(descs)[:nb * 32]), dtype=torch.uint8).to(dev)
    d_out = torch.zeros(nb * info.block_max, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(nb * 32, dtype=torch.uint8, device=dev)
    lz4ada.decode_blocks_device(d_frame.data_ptr(), len(frame), d_desc.data_ptr(), nb,
                                d_out.data_ptr(), d_st.data_ptr(),
                                torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    st = (lz4ada.BlockStatus * nb).from_buffer_copy(d_st.cpu().numpy().tobytes())
    out = d_out.cpu().numpy().tobytes()
    for i in range(nb):
        assert st[i].code == 0 and st[i].out_len == descs[i].in_len
        assert st[i].cksum == descs[i].cksum, i
        o = descs[i].out_off
        assert out[o:o + st[i].out_len] == blocks[i][1]
    # a corrupted stored block: the reference's checksum error, at that block
    bad = bytearray(frame)
    bad[descs[nblocks // 2].in_off + 3] ^= 0x40
    with pytest.raises(lz4ada.ChecksumError) as ei:
        lz4ada.decode_frame(bytes(bad))
    stx, msg = O.error_harness(bytes(bad))
    assert str(ei.value) == O.exception_information(stx, msg)
