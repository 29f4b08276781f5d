"""The literal-heavy decoder (k_decode_sparse, lz4ada_sparse.hip) against the
oracle: blocks pass 1 declines as sparse decode byte-exactly through it
alone (variant IDX_SPARSE: no two-wave retry), and anything it must not
take -- malformed data, a reference before the block start, a chain that
turns dense -- is declined and then decoded exactly by the full chain."""
import random

import pytest

import _lz4build as B
import _oracle as O
import lz4ada
import lz4frame

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not lz4ada.device_available():
        pytest.fail("MI355X not usable: " + lz4ada._thread_error())


def run_variant(frame, variant):
    import torch
    info, descs = lz4ada.frame_index(frame)
    nb, bmax = info.nblocks, info.block_max
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
    out = d_out.cpu().numpy().tobytes()
    return info, st, [out[i * bmax:i * bmax + st[i].out_len] for i in range(nb)]


def sparse_blocks(seed, sizes, end_after_match=()):
    rng = random.Random(seed)
    blocks = []
    for i, n in enumerate(sizes):
        seqs = B.sparse_seqs(rng, n)
        fin = None if i in end_after_match else rng.randbytes(rng.randint(12, 700))
        blocks.append(B.encode(seqs, fin))
    return blocks


@pytest.mark.parametrize("bmax,sizes", [
    (4 << 20, [(4 << 20) - 5000, (4 << 20) - 3000, 300_000, 70_000]),
    (256 << 10, [250_000, 200_000, 240_000, 100_000]),
])
def test_sparse_alone_exact(bmax, sizes):
    blocks = sparse_blocks(11, sizes, end_after_match=(1,))
    assert all(len(r) <= bmax for _, r in blocks)
    frame, raw = lz4frame.build_frame([(c, r, False) for c, r in blocks], bmax, block_cksum=True)
    st0, want, _, msg = O.decode_stream(frame)
    assert st0 == O.OK and want == raw, msg
    info, st, outs = run_variant(frame, lz4ada.DECODE_IDX_SPARSE)
    for i, (c, r) in enumerate(blocks):
        assert st[i].code == 0, (i, st[i].code)  # taken by the sparse decoder itself
        assert outs[i] == r, i
    out, _ = lz4ada.decode_frame(frame)
    assert out == raw


def test_sparse_long_runs_exact():
    """Literal runs longer than the staged window (copied HBM -> HBM, the
    staging stream restarted past them) mixed with short ones."""
    rng = random.Random(5)
    bmax = 4 << 20
    blocks = []
    for n, lo, hi in [((4 << 20) - 40000, 1500, 30000), (2 << 20, 40, 9000), (600_000, 3000, 70000)]:
        seqs = B.sparse_seqs(rng, n, lit_lo=lo, lit_hi=hi)
        blocks.append(B.encode(seqs, rng.randbytes(rng.randint(12, 5000))))
    assert all(len(r) <= bmax for _, r in blocks)
    frame, raw = lz4frame.build_frame([(c, r, False) for c, r in blocks], bmax, block_cksum=True)
    st0, want, _, msg = O.decode_stream(frame)
    assert st0 == O.OK and want == raw, msg
    info, st1, _ = run_variant(frame, lz4ada.DECODE_IDX_ALONE)
    sp = [i for i in range(len(blocks)) if st1[i].code == lz4ada.DS_SPARSE]
    assert len(sp) >= 2, [s.code for s in st1[:len(blocks)]]  # pass 1 hands them over
    info, st, outs = run_variant(frame, lz4ada.DECODE_IDX_SPARSE)
    for i in sp:
        assert st[i].code == 0, (i, st[i].code, st[i].detail, st[i].err_out_pos)
        assert outs[i] == blocks[i][1], i
    out, _ = lz4ada.decode_frame(frame)
    assert out == raw


def test_literal_class_taken_by_sparse():
    """The bench's literal class (4 MiB blocks) is pass 1's sparse case and
    k_decode_sparse's whole job."""
    bmax = 4 << 20
    blocks = [lz4ada.gen_block(lz4ada.GEN_LITERAL, 0x4C5A3441 + i, bmax) for i in range(4)]
    frame, raw = lz4frame.build_frame([(c, r, False) for c, r in blocks], bmax, block_cksum=True)
    info, st, outs = run_variant(frame, lz4ada.DECODE_IDX_ALONE)
    assert all(s.code == lz4ada.DS_SPARSE for s in st[:4])
    info, st, outs = run_variant(frame, lz4ada.DECODE_IDX_SPARSE)
    for i, (c, r) in enumerate(blocks):
        assert st[i].code == 0 and outs[i] == r, i


@pytest.mark.parametrize("bmax", [4 << 20, 64 << 10])
def test_rle_class_taken_by_sparse(bmax):
    """RLE blocks (at least 4 KiB of input and more than 64 output bytes per
    input byte; runs of 255-bytes in the match-length extensions, on which
    pass 1's speculative walks would crawl) are handed to the scalar-parse
    decoder before any walk; its whole-wave pattern fills write them."""
    blocks = [lz4ada.gen_block(lz4ada.GEN_RLE, 0x4C5A3441 + i, bmax) for i in range(3)]
    frame, raw = lz4frame.build_frame([(c, r, False) for c, r in blocks], bmax, block_cksum=True)
    info, st, outs = run_variant(frame, lz4ada.DECODE_IDX_ALONE)
    if bmax == 4 << 20:  # (short RLE blocks, under 4 KiB of input, stay with pass 1)
        assert all(s.code == lz4ada.DS_SPARSE for s in st[:3]), [s.code for s in st[:3]]
    info, st, outs = run_variant(frame, lz4ada.DECODE_IDX_SPARSE)
    for i, (c, r) in enumerate(blocks):
        if st[i].code == 0:
            assert outs[i] == r, i
    assert lz4ada.decode_frame(frame)[0] == raw


def _with_fault(kind):
    rng = random.Random(23)
    seqs = B.sparse_seqs(rng, 1 << 20)
    k = 600 if kind != "pre_block" else 60  # (pre_block: within the first 64 KiB)
    lits, off, ml = seqs[k]
    if kind == "offset0":
        seqs[k] = (lits, 0, ml)
    elif kind == "pre_block":  # D2: reads before the block start
        pos = sum(len(a) + m for a, _, m in seqs[:k]) + len(lits)
        seqs[k] = (lits, min(pos + 1, 65535), ml)
    comp, raw = B.encode(seqs, rng.randbytes(100))
    if kind == "dense_tail":
        dense_c, dense_r = lz4ada.gen_block(lz4ada.GEN_DENSE, 5, 1 << 20)
        # a literal-only sparse head cannot precede a dense chain in one
        # block, so splice: sparse sequences, then the dense block's
        # sequences (its first one has literals only where it starts at 0)
        comp, raw = B.encode(seqs, None)
        comp += dense_c
        raw += dense_r
    return comp, raw


@pytest.mark.parametrize("kind", ["offset0", "pre_block", "dense_tail"])
def test_sparse_declines_then_exact(kind):
    comp, raw = _with_fault(kind)
    bmax = 4 << 20
    frame, _ = lz4frame.build_frame([(comp, raw, False)], bmax, block_cksum=True)
    info, st, _ = run_variant(frame, lz4ada.DECODE_IDX_ALONE)
    assert st[0].code == lz4ada.DS_SPARSE
    info, st, _ = run_variant(frame, lz4ada.DECODE_IDX_SPARSE)
    assert st[0].code == lz4ada.DS_RETRY  # declined, nothing claimed
    info, st_full, outs = run_variant(frame, lz4ada.DECODE_IDX)
    info, st_pc, outs_pc = run_variant(frame, lz4ada.DECODE_PC)
    assert (st_full[0].code, st_full[0].out_len) == (st_pc[0].code, st_pc[0].out_len)
    assert outs == outs_pc
    if kind == "dense_tail":
        assert st_full[0].code == 0 and outs[0] == raw
    # the product's answer is the reference's (output or exception text)
    ost, oref, _, omsg = O.decode_stream(frame)
    if ost == O.OK:
        assert lz4ada.decode_frame(frame)[0] == oref
    else:
        with pytest.raises(lz4ada.LZ4AdaError) as ei:
            lz4ada.decode_frame(frame)
        assert str(ei.value) == O.exception_information(ost, omsg)
