"""GPU parity of the linked-frame bulk path (lz4ada_linked.hip),
the bounded-slot bulk path for independent frames, and the bulk API's
error behaviour, against the CPU oracle (oracle/lz4ada_oracle.c, the C
restatement of lib/lz4ada.adb).

The reference decodes every frame as linked (B.Indep is never read,
lz4ada.adb:267-275): a block's matches may read the 64 KiB before it.  The
bulk path decodes every block at once against synthetic history and
resolves the history bytes on the GPU; it hands the frame to the exact path
when the reference would diverge from contiguous history (quirk D1) or
raise.  lz4ada.last_path() says which path ran, so the tests check both the
bytes and that the fast path really took them.
"""
import os
import random
import struct

import pytest

import _oracle as O
from conftest import error_vectors, good_vectors, read_eds, read_vector

import lz4ada
import lz4frame

pytestmark = pytest.mark.gpu

KiB = 1024


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not lz4ada.device_available():
        pytest.fail("MI355X not usable: " + lz4ada._thread_error())


@pytest.fixture
def env():
    """Set environment knobs of the library for one test."""
    saved = {}

    def set_(k, v):
        saved.setdefault(k, os.environ.get(k))
        os.environ[k] = v
    yield set_
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def linked_frame(kind, lens, bmax, seed=0x4C5A3441, block_cksum=True, content_cksum=True,
                 content_size=False, indep=False):
    blocks = lz4ada.gen_linked_blocks(kind, seed, 0, 0, lens=lens)
    frame, raw = lz4frame.build_frame([(c, r, False) for c, r in blocks], bmax, indep=indep,
                                      block_cksum=block_cksum, content_cksum=content_cksum,
                                      with_content_size=content_size)
    return frame, raw, blocks


def oracle(frame):
    st, out, msg = O.unlz4ada(frame, out_cap=4 * len(frame) + (64 << 20))
    return st, out, msg


def same_as_oracle(frame, decode=lambda f: lz4ada.decode_frame(f)[0]):
    """decode(frame) gives the oracle's output, or raises its exception."""
    st, ref, msg = oracle(frame)
    if st == O.OK:
        assert decode(frame) == ref
    else:
        with pytest.raises(lz4ada.LZ4AdaError) as ei:
            decode(frame)
        assert str(ei.value) == O.exception_information(st, msg)
    return st, ref


def matches(payload):
    """(output position, offset) of every match of an LZ4 block (test-side
    parse of the block format, lz4ada.adb:737-777)."""
    i, o, n = 0, 0, len(payload)
    while i < n:
        t = payload[i]
        i += 1
        lit = t >> 4
        if lit == 15:
            while True:
                b = payload[i]
                i += 1
                lit += b
                if b != 255:
                    break
        i += lit
        o += lit
        if i >= n:
            break
        off = payload[i] | (payload[i + 1] << 8)
        i += 2
        ml = t & 15
        if ml == 15:
            while True:
                b = payload[i]
                i += 1
                ml += b
                if b != 255:
                    break
        yield o, off
        o += ml + 4


def d1_matches(payload, n1, oph):
    """(L, lit, match output position, offset, ml, previous match) of the
    block's matches in quirk D1's domain for round state (n1, oph): a read
    before the round start within 7 bytes of where the last round ended.
    The previous match is (output position, offset, ml), None for the
    block's first sequence."""
    i, o, n = 0, 0, len(payload)
    prev = None
    while i < n:
        t = payload[i]
        i += 1
        L = t >> 4
        if L == 15:
            while True:
                b = payload[i]
                i += 1
                L += b
                if b != 255:
                    break
        lit = i
        i += L
        if i >= n:
            return
        off = payload[i] | (payload[i + 1] << 8)
        i += 2
        ml = t & 15
        if ml == 15:
            while True:
                b = payload[i]
                i += 1
                ml += b
                if b != 255:
                    break
        ml += 4
        m = o + L
        if n1 + m < off and oph - off < 8:
            yield L, lit, m, off, ml, prev
        prev = (m, off, ml)
        o = m + ml


def d1_emulable(payload, n1, oph):
    """Whether the index decoder emulates every D1 read of the block under
    round state (n1, oph) (lz4ada_idx.hip d1_emulable).  A read without
    literals copies the bytes after the previous match's source (from HBM,
    or as a ring copy of its own when they are recent)."""
    for L, lit, m, off, ml, prev in d1_matches(payload, n1, oph):
        if n1 + m + ml > off:
            return False
        if L > 0:
            if lit + 8 * ((L - 1) // 8) + 8 > len(payload):
                return False
            continue
        if prev is None:
            if n1 + m != 0:
                return False
            continue  # the round's first output: plain history
        pm, po, pml = prev
        f, pad = n1 + pm, (8 - pml % 8) % 8
        raw = f - po
        ok = (pml <= po and po - pml >= pad) if raw >= 0 else \
            (po - f >= pml and oph - po >= 8 and raw + pml + pad <= 0)
        if not ok:
            return False
    return True


def batch_starts(blocks, bmax, budget):
    """Block indices where lz4ada_bulk_linked.cpp's batches start (batches_of:
    each block's slot, rounded to 256 bytes, plus its 64 KiB history region;
    at least one block a batch)."""
    starts, acc = [0], 0
    for k, (comp, raw) in enumerate(blocks):
        need = ((min(bmax, 255 * len(comp) + 64) + 255) & ~255) + 65536
        if k > starts[-1] and acc + need > budget:
            starts.append(k)
            acc = 0
        acc += need
    return set(starts)


def d1_stop(blocks, bmax, budget=None):
    """The first block the linked bulk path hands to the exact path for
    quirk D1 (lz4ada_bulk_linked.cpp bulk_linked), or None.  The host
    predicts each block's round state (Output_Pos / Output_Pos_History,
    lz4ada.adb:678-690, 785-787) with every block filling its slot; the
    index decoder emulates D1 under the prediction where d1_emulable says so
    (else it declines the block, and k_decode_pc decodes it without
    emulation).  A block with a match >= 65529 back before its start goes
    exact when it is in a D1 round and was not emulated under the real
    state, or when it was emulated under a D1 prediction the real state
    lacks.  Predictions restart from the real state at every batch
    (LZ4ADA_LINKED_BATCH_BYTES)."""
    budget = budget or int(os.environ.get("LZ4ADA_LINKED_BATCH_BYTES", 2 << 30))
    starts = batch_starts(blocks, bmax, budget)
    opos = oph = po = ph = 0
    for k, (comp, raw) in enumerate(blocks):
        if k in starts:  # each batch predicts from the real state at its start
            po, ph = opos, oph
        if opos >= 65536:
            opos = 0
        if po >= 65536:
            po = 0
        risk = any(off > q and off >= 65529 for q, off in matches(comp))
        in_d1, pd1 = 65536 <= oph <= 65542, 65536 <= ph <= 65542
        emu = pd1 and d1_emulable(comp, po, ph)
        if risk and (not (emu and (po, ph) == (opos, oph)) if in_d1 else emu):
            return k
        opos += len(raw)
        po += min(bmax, 255 * len(comp) + 64)
        if opos >= 65536:
            oph = opos
        if po >= 65536:
            ph = po
    return None


def want_path(blocks, bmax, ok=True):
    """The path lz4ada_last_path() reports: the linked bulk path takes the
    frame; at a block quirk D1 sends to the exact path, that path resumes
    and finishes it.  ok=False (the reference raises at the end, e.g. a
    content checksum its D1 bytes do not match): a bulk pass that reaches
    the end hands the whole frame to the exact path for the exception."""
    L, E = lz4ada.PATH_LINKED, lz4ada.PATH_EXACT
    return L | E if d1_stop(blocks, bmax) is not None else (L if ok else E)


# ------------------------------------------------------------ linked frames

@pytest.mark.parametrize("kind", ["dense", "mixed", "literal", "chain"])
@pytest.mark.parametrize("bmax", [64 * KiB, 256 * KiB, 1 << 20, 4 << 20])
def test_linked_frame_bulk(kind, bmax):
    nb = {64 * KiB: 12, 256 * KiB: 6, 1 << 20: 4, 4 << 20: 3}[bmax]
    lens = [bmax] * (nb - 1) + [bmax // 3 + 11]
    frame, raw, blocks = linked_frame(lz4ada.GEN_KINDS[kind], lens, bmax)
    st, ref, msg = oracle(frame)
    if st == O.OK:
        out, consumed = lz4ada.decode_frame(frame)
        assert consumed == len(frame)
        assert out == ref
    else:
        # 64 KiB dense: the reference's D1 overshoot really corrupts the
        # history, and the content checksum catches it
        with pytest.raises(lz4ada.LZ4AdaError) as ei:
            lz4ada.decode_frame(frame)
        assert str(ei.value) == O.exception_information(st, msg)
    assert lz4ada.last_path() == want_path(blocks, bmax, st == O.OK)


def test_linked_frame_mixed_block_sizes():
    """Short blocks anywhere (history spans several blocks), declared content
    size, block and content checksums."""
    lens = [5000, 65536, 100, 70000, 1, 200000, 65536, 65536, 30000, 262144, 17]
    frame, raw, blocks = linked_frame(lz4ada.GEN_MIXED, lens, 256 * KiB, seed=99,
                                      content_size=True)
    st, ref, msg = oracle(frame)
    assert st == O.OK and ref == raw, msg
    out, _ = lz4ada.decode_frame(frame)
    assert out == raw
    assert lz4ada.last_path() == want_path(blocks, 256 * KiB)


@pytest.mark.parametrize("batch", [None, 300 * KiB, 1])
def test_linked_pointer_chains_through_every_block(batch, env):
    """`chain` data: every block copies the previous block's tail, so each
    history byte resolves through every earlier block (pointer jumping,
    ~log2 rounds); small batches carry the real 64 KiB tail across."""
    if batch:
        env("LZ4ADA_LINKED_BATCH_BYTES", str(batch))
    lens = [100000] * 40 + [777]
    frame, raw, blocks = linked_frame(lz4ada.GEN_CHAIN, lens, 256 * KiB, seed=5)
    st, ref, msg = oracle(frame)
    assert st == O.OK and ref == raw, msg
    out, _ = lz4ada.decode_frame(frame)
    assert out == raw
    assert lz4ada.last_path() == lz4ada.PATH_LINKED


@pytest.mark.parametrize("batch", [None, 300 * KiB])
@pytest.mark.parametrize("words", ["full", "sparse"])
@pytest.mark.parametrize("kind", ["dense", "mixed", "chain"])
def test_linked_word_modes(kind, words, batch, env):
    """Both ways k_link_init leaves the words (lz4ada_bulk_linked.cpp picks
    one from the z decoder's history count; LZ4ADA_LINK_WORDS forces it):
    every word, or words only where a byte is still open plus the map of
    final bytes, and the rounds after it -- over ragged block lengths, and
    in small batches, where init's steps and the rounds read the previous
    batch's tail for sources before the batch."""
    env("LZ4ADA_LINK_WORDS", words)
    if batch:
        env("LZ4ADA_LINKED_BATCH_BYTES", str(batch))
    lens = [65536, 70001, 100, 65535, 131075, 3, 65536, 200001, 4097]
    frame, raw, blocks = linked_frame(lz4ada.GEN_KINDS[kind], lens, 256 * KiB, seed=17)
    st, _ = same_as_oracle(frame)
    assert lz4ada.last_path() == want_path(blocks, 256 * KiB, st == O.OK)


def test_linked_small_batches_64k(env):
    env("LZ4ADA_LINKED_BATCH_BYTES", str(200 * KiB))
    frame, raw, blocks = linked_frame(lz4ada.GEN_MIXED, [65536] * 9 + [4000], 64 * KiB, seed=3)
    st, _ = same_as_oracle(frame)
    assert lz4ada.last_path() == want_path(blocks, 64 * KiB, st == O.OK)


def d1_frame(content_cksum):
    """a full 64 KiB block (Output_Pos_History = 65536),
    then a block whose 20-byte literal run is followed by a match of offset
    65533: the reference's 8-byte wild copy of the literals has already
    overwritten history bytes 21..23 that the match reads."""
    comp0, raw0 = lz4ada.gen_block(1, 1234, 65536)
    lits = bytes(range(65, 85))
    tail = b"vwxyz"
    comp1 = bytes([0xF6, 20 - 15]) + lits + struct.pack("<H", 65533) + bytes([0x50]) + tail
    spec1 = lits + raw0[23:33] + tail  # contiguous history (liblz4 semantics)
    frame, spec = lz4frame.build_frame([(comp0, raw0, False), (comp1, spec1, False)], 64 * KiB,
                                       indep=False, content_cksum=content_cksum)
    return frame, spec


def test_d1_emulated_in_bulk_matches_reference():
    frame, spec = d1_frame(content_cksum=False)
    st, ref, msg = oracle(frame)
    assert st == O.OK, msg
    assert ref != spec  # the reference really diverges here
    out, _ = lz4ada.decode_frame(frame)
    assert out == ref
    # both blocks through the linked bulk path: block 1's D1 match emulated
    # under the predicted round state (Output_Pos_History 65536, Output_Pos 0)
    assert lz4ada.last_path() == lz4ada.PATH_LINKED


def test_d1_uniform_offsets_64k_frame():
    """LZ4F's default block mode (64 KiB linked) with uniform match offsets:
    quirk D1 in ~1 block of 6 (tools/d1_frame_time.py's frame).  Emulated
    in bulk, with the exact path only from the first block the decoder
    cannot emulate; the bytes are the reference's."""
    blocks = lz4ada.gen_linked_blocks(lz4ada.GEN_MIXED, 0x4C5A3441, 64 * KiB, 64)
    frame, _ = lz4frame.build_frame([(c, r, False) for c, r in blocks], 64 * KiB, indep=False)
    st, ref, msg = oracle(frame)
    assert st == O.OK, msg
    out, _ = lz4ada.decode_frame(frame)
    assert out == ref
    assert lz4ada.last_path() == want_path(blocks, 64 * KiB)


@pytest.mark.parametrize("lit_len,pof,pml,off", [(16, 16, 4, 65533), (16, 16, 9, 65535), (3, 1000, 10, 65534),
                                                 (3, 40000, 4, 65535), (3, 20, 9, 65530)])
def test_d1_without_literals_in_bulk(lit_len, pof, pml, off):
    """Quirk D1 right after a match (test_gpu_facade.py's d1_frame_l0
    shapes) through the linked bulk path: the previous match's source tail
    from the history region (HBM) or from this batch's output (a ring copy
    of its own in k_decode_idx_lk); the reference's bytes, no exact path."""
    from test_gpu_facade import d1_frame_l0
    frame = d1_frame_l0(lit_len, pof, pml, off)
    st, ref, msg = oracle(frame)
    assert st == O.OK, msg
    out, _ = lz4ada.decode_frame(frame)
    assert out == ref
    info, descs = lz4ada.frame_index(frame)
    blocks = [(frame[d.in_off:d.in_off + d.in_len], b"\0" * (65536 if k == 0 else len(ref) - 65536))
              for k, d in enumerate(descs[:info.nblocks])]
    assert lz4ada.last_path() == want_path(blocks, 64 * KiB)
    assert lz4ada.last_path() == lz4ada.PATH_LINKED


@pytest.mark.parametrize("off,ml", [(65529, 4), (65533, 10), (65535, 40)])
def test_d1_as_first_output_in_bulk(off, ml):
    """A D1-range read as the round's first output (test_gpu_facade.py's
    d1_frame_first): plain history, the whole frame on the bulk path."""
    from test_gpu_facade import d1_frame_first
    frame = d1_frame_first(off, ml)
    st, ref, msg = oracle(frame)
    assert st == O.OK, msg
    out, _ = lz4ada.decode_frame(frame)
    assert out == ref
    assert lz4ada.last_path() == lz4ada.PATH_LINKED


def test_d1_with_content_checksum_raises_like_reference():
    frame, spec = d1_frame(content_cksum=True)
    st, ref, msg = oracle(frame)
    assert st == O.CHECKSUM_ERROR, msg
    with pytest.raises(lz4ada.ChecksumError) as ei:
        lz4ada.decode_frame(frame)
    assert str(ei.value) == O.exception_information(st, msg)


@pytest.mark.parametrize("where", ["first", "second"])
def test_reference_before_frame_start(where):
    """A match reading before the frame start: the reference's
    'Backreference location out of range' (lz4ada.adb:867-874)."""
    bad = bytes([0x14]) + b"A" + struct.pack("<H", 5) + bytes([0x50]) + b"abcde"
    blocks = []
    if where == "second":
        comp, raw = lz4ada.gen_block(1, 7, 3000)
        blocks.append((comp, raw, False))
        bad = bytes([0x14]) + b"A" + struct.pack("<H", 3010) + bytes([0x50]) + b"abcde"
    blocks.append((bad, b"", False))
    frame, _ = lz4frame.build_frame(blocks, 64 * KiB, indep=False)
    st, ref, msg = oracle(frame)
    assert st == O.DATA_CORRUPTION, msg
    with pytest.raises(lz4ada.DataCorruption) as ei:
        lz4ada.decode_frame(frame)
    assert str(ei.value) == O.exception_information(st, msg)


def test_independent_flag_with_cross_block_refs_uses_linked_path():
    """D2: B.Indep set, but blocks read earlier blocks.  The reference ignores
    the flag; the bulk path detects the references and resolves them."""
    frame, raw, blocks = linked_frame(lz4ada.GEN_MIXED, [256 * KiB] * 4 + [999], 256 * KiB,
                                      indep=True)
    st, ref, msg = oracle(frame)
    assert st == O.OK and ref == raw, msg
    out, _ = lz4ada.decode_frame(frame)
    assert out == raw
    assert lz4ada.last_path() == lz4ada.PATH_LINKED


@pytest.mark.parametrize("kind", ["dense", "mixed", "rle", "literal"])
def test_forced_linked_path_on_independent_frames(kind, env):
    """The linked machinery on independent data (stored blocks included)."""
    env("LZ4ADA_FORCE_LINKED", "1")
    rng = random.Random(11)
    blocks = []
    for i in range(7):
        n = 64 * KiB if i < 6 else 1234
        if i == 3:
            raw = rng.randbytes(n)
            blocks.append((raw, raw, True))
        else:
            comp, raw = lz4ada.gen_block(lz4ada.GEN_KINDS[kind], 50 + i, n)
            blocks.append((comp, raw, False))
    frame, raw = lz4frame.build_frame(blocks, 64 * KiB, block_cksum=True, content_cksum=True)
    out, _ = lz4ada.decode_frame(frame)
    assert out == raw
    assert lz4ada.last_path() == lz4ada.PATH_LINKED


@pytest.mark.parametrize("what", ["block_cksum", "content_cksum", "content_size"])
def test_linked_frame_errors_match_reference(what):
    lens = [256 * KiB] * 3 + [5000]
    blocks = lz4ada.gen_linked_blocks(lz4ada.GEN_MIXED, 21, 0, 0, lens=lens)
    raw = b"".join(r for _, r in blocks)
    hdr = lz4frame.header(256 * KiB, indep=False, block_cksum=True, content_cksum=True,
                          content_size=len(raw) + (7 if what == "content_size" else 0))
    recs = [lz4frame.block_record(c, block_cksum=True) for c, _ in blocks]
    if what == "block_cksum":
        r = bytearray(recs[2])
        r[100] ^= 1
        recs[2] = bytes(r)
    h = lz4frame.xxhash.xxh32(raw).intdigest() ^ (1 if what == "content_cksum" else 0)
    frame = hdr + b"".join(recs) + lz4frame.trailer(content_cksum=True, content_hash=h)
    st, ref, msg = oracle(frame)
    assert st != O.OK
    with pytest.raises(lz4ada.LZ4AdaError) as ei:
        lz4ada.decode_frame(frame)
    assert str(ei.value) == O.exception_information(st, msg)


def test_linked_device_api():
    """lz4ada_decode_linked_device: device-resident frame -> contiguous output."""
    import torch
    frame, raw, _ = linked_frame(lz4ada.GEN_DENSE, [256 * KiB] * 5 + [3333], 256 * KiB)
    info, descs = lz4ada.frame_index(frame)
    d_frame = torch.frombuffer(bytearray(frame), dtype=torch.uint8).cuda()
    d_out = torch.empty(len(raw) + 16, dtype=torch.uint8, device="cuda")
    n = lz4ada.decode_linked_device(d_frame.data_ptr(), len(frame), descs, info.nblocks,
                                    info.block_max, d_out.data_ptr(), len(raw) + 16)
    assert n == len(raw)
    assert bytes(d_out[:n].cpu().numpy()) == raw
    with pytest.raises(lz4ada.NeedsExactPath):
        lz4ada.decode_linked_device(d_frame.data_ptr(), len(frame), descs, info.nblocks,
                                    info.block_max, d_out.data_ptr(), len(raw) - 1)


# ------------------------------------------- bounded slots, independent frames

@pytest.mark.parametrize("batch", [None, 1 << 16])
def test_many_small_blocks_under_a_4mib_bd(batch, env):
    """Thousands of small (flushed) blocks under BD = 4 MiB: slots are sized
    from each block's bound, not block_max (that would be ~12 GiB here)."""
    if batch:
        env("LZ4ADA_BATCH_BYTES", str(batch))
    rng = random.Random(4)
    blocks = []
    for i in range(3000):
        comp, raw = lz4ada.gen_block(i % 4, 1000 + i, rng.randint(1, 600))
        blocks.append((comp, raw, False))
    frame, raw = lz4frame.build_frame(blocks, 4 << 20, block_cksum=True, content_cksum=True)
    out, _ = lz4ada.decode_frame(frame)
    assert out == raw
    assert lz4ada.last_path() == lz4ada.PATH_INDEPENDENT


# ------------------------------------------------ bulk API on bad input

@pytest.mark.parametrize("name", error_vectors())
def test_bulk_api_on_error_vectors(name):
    """decode_frame raises the exact .eds line of every .err vector (the
    reference's Init_With_Header(Single_Frame) + Update harness,
    lz4test.adb:280-351) -- no output bound is needed up front any more --
    and decode_stream raises what the unlz4ada loop raises."""
    data = read_vector(name, "err")
    if name == "trailingbytes":
        # one frame, then bytes after its end mark: decode_frame returns
        # that frame and how much it consumed (the caller sees the rest)
        out, consumed = lz4ada.decode_frame(data)
        assert consumed < len(data)
    else:
        with pytest.raises(lz4ada.LZ4AdaError) as ei:
            lz4ada.decode_frame(data)
        assert str(ei.value) == read_eds(name)
    st, ref, msg = oracle(data)
    assert st != O.OK
    with pytest.raises(lz4ada.LZ4AdaError) as ei:
        lz4ada.decode_stream(data)
    assert str(ei.value) == O.exception_information(st, msg)


@pytest.mark.parametrize("name", [n for n in good_vectors() if n not in ("z9m", "b3444k")])
def test_bulk_api_on_truncated_vectors(name):
    data = read_vector(name, "lz4")
    for cut in sorted({7, len(data) // 2, len(data) - 5, len(data) - 1}):
        if cut <= 0 or cut >= len(data):
            continue
        piece = data[:cut]
        st, ref, msg = oracle(piece)
        if st == O.OK:
            assert lz4ada.decode_stream(piece) == ref, cut
        else:
            with pytest.raises(lz4ada.LZ4AdaError) as ei:
                lz4ada.decode_stream(piece)
            assert str(ei.value) == O.exception_information(st, msg), cut
