"""The lone-block decoder (lz4ada_lone.hip: one block by the whole GPU, the
streaming facade's decoder) against the generator's bytes and the CPU
oracle's block decode (oracle/lz4ada_oracle.c, lz4ada.adb:716-904): every
block it accepts is byte-exact; anything the reference would reject or that
reads before the block start is declined (status 10), never decoded
differently."""
import ctypes
import random

import pytest

import _oracle as O
from _lz4build import encode, sparse_seqs

import lz4ada

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not lz4ada.device_available():
        pytest.fail("MI355X not usable: " + lz4ada._thread_error())


def run_lone(comp, cap):
    import torch
    n = len(comp)
    d_in = torch.frombuffer(bytearray(comp + b"\0" * 16), dtype=torch.uint8).cuda()
    d_out = torch.zeros(max(cap, 1), dtype=torch.uint8, device="cuda")
    d_st = torch.zeros(ctypes.sizeof(lz4ada.BlockStatus), dtype=torch.uint8, device="cuda")
    sb = lz4ada.lone_scratch_bytes(n, cap)
    d_sc = torch.empty(sb, dtype=torch.uint8, device="cuda")
    lz4ada.launch_decode_lone(d_in.data_ptr(), n, d_out.data_ptr(), cap, d_st.data_ptr(),
                              d_sc.data_ptr(), sb, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    st = lz4ada.BlockStatus.from_buffer_copy(d_st.cpu().numpy().tobytes())
    return st, d_out[:st.out_len].cpu().numpy().tobytes() if st.code == 0 else b""


def oracle_block(comp, cap):
    """(ok, bytes) of the reference decoding comp as one raw block."""
    ctx = O.Decompressor.init_for_block(len(comp))
    buf = ctypes.create_string_buffer(ctx.min_buffer_size)
    st, c, f, l = ctx.update(comp, buf)
    if st != O.OK:
        return False, b""
    out = buf.raw[f:l + 1] if l >= f else b""
    return len(out) <= cap, out


@pytest.mark.parametrize("kind", ["dense", "mixed", "rle", "literal"])
@pytest.mark.parametrize("size", [1, 13, 100, 511, 512, 513, 1023, 1024, 1025, 2047, 2049, 4095, 4096,
                                  4097, 65536, 200001, 300001, 1 << 20, 3 << 20, 4 << 20])
def test_lone_generated_blocks(kind, size):
    comp, raw = lz4ada.gen_block(lz4ada.GEN_KINDS[kind], 0x10E + size, size)
    st, out = run_lone(comp, 4 << 20)
    assert st.code == 0, st.code
    assert st.out_len == len(raw)
    assert out == raw


@pytest.mark.parametrize("seed", range(6))
def test_lone_long_literals_and_matches(seed):
    """Runs longer than a 4 KiB window (a sequence jumping over windows),
    one-byte and multi-byte length extensions, overlapping matches."""
    rng = random.Random(seed)
    seqs = sparse_seqs(rng, 3 << 20, lit_lo=1, lit_hi=20000,
                       offs=[1, 2, 3, 7, 16, 100, 5000, 60000], mls=[4, 18, 19, 300, 70000])
    comp, raw = encode(seqs, final_lits=rng.randbytes(rng.choice([0, 5, 40])))
    st, out = run_lone(comp, 4 << 20)
    assert st.code == 0, st.code
    assert out == raw


def test_lone_output_over_cap_declines():
    comp, raw = lz4ada.gen_block(lz4ada.GEN_MIXED, 5, 1 << 20)
    st, _ = run_lone(comp, len(raw) - 1)
    assert st.code == lz4ada.DS_RETRY
    st, out = run_lone(comp, len(raw))
    assert st.code == 0 and out == raw


def test_lone_reference_before_block_start_declines():
    blocks = lz4ada.gen_linked_blocks(lz4ada.GEN_MIXED, 3, 0, 0, lens=[65536, 65536])
    st, _ = run_lone(blocks[1][0], 1 << 20)
    assert st.code == lz4ada.DS_RETRY


@pytest.mark.parametrize("seed", range(24))
def test_lone_corrupted_blocks_never_differ(seed):
    rng = random.Random(seed)
    comp, raw = lz4ada.gen_block(seed % 4, 77 + seed, rng.choice([5000, 70000, 300000]))
    b = bytearray(comp)
    for _ in range(rng.randrange(1, 4)):
        b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
    if seed % 5 == 0:
        b = b[:rng.randrange(1, len(b))]
    cap = 1 << 20
    ok, ref = oracle_block(bytes(b), cap)
    st, out = run_lone(bytes(b), cap)
    assert st.code in (0, lz4ada.DS_RETRY)
    if st.code == 0:
        assert ok and out == ref


# ------------------------------------------- frames of a few large blocks
# (lz4ada_host_common.h few_large_blocks: decode_frame and the facade's read-ahead
# take such frames one block at a time through the lone-block decoder)

def few_block_frame(kinds, seed=9, stored_at=None):
    import lz4frame
    blocks = []
    for i, k in enumerate(kinds):
        if i == stored_at:
            raw = random.Random(seed + i).randbytes(3 << 20)
            blocks.append((raw, raw, True))
        else:
            comp, raw = lz4ada.gen_block(lz4ada.GEN_KINDS[k], seed * 100 + i, 4 << 20)
            blocks.append((comp, raw, False))
    return lz4frame.build_frame(blocks, 4 << 20, indep=True, block_cksum=True, content_cksum=True)


@pytest.mark.parametrize("kinds,stored_at", [
    (["mixed"] * 5, None),
    (["literal", "dense", "mixed", "rle"], 2),
])
def test_few_large_blocks_decode_frame(kinds, stored_at):
    frame, raw = few_block_frame(kinds, stored_at=stored_at)
    out, cons = lz4ada.decode_frame(frame)
    assert out == raw and cons == len(frame)
    assert lz4ada.last_path() == lz4ada.PATH_INDEPENDENT


def test_few_large_blocks_bad_checksum_is_the_references():
    frame, raw = few_block_frame(["mixed"] * 4)
    info, descs = lz4ada.frame_index(frame)
    b = bytearray(frame)
    b[descs[2].in_off + 999] ^= 4
    st, ref, msg = O.unlz4ada(bytes(b), out_cap=len(raw) + (1 << 20))
    out, cons, exc = lz4ada.decode_frame_partial(bytes(b))
    assert exc is not None and str(exc) == O.exception_information(st, msg)
    assert out == ref


def test_few_large_blocks_facade_read_ahead():
    frame, raw = few_block_frame(["mixed", "dense", "literal"])
    ctx, used, mbs = lz4ada.Decompressor.init_with_header(frame)
    buf = bytearray(mbs)
    out, pos = bytearray(), used
    while pos < len(frame):
        c, f, l = ctx.update(frame, buf, pos)  # all remaining input each call
        if l >= f:
            out += buf[f:l + 1]
        pos += c
        if ctx.is_end_of_frame() == lz4ada.EndOfFrame.Yes:
            break
    assert bytes(out) == raw


def test_lone_input_limit_refused_and_facade_exact():
    """A block over LONE_MAX_IN (16 MiB compressed: the chain step holds
    every window's entry in one workgroup) is refused by the launcher
    instead of decoded with windows missing, and the facade
    sends it to the exact path (Init_For_Block, lz4ada.ads:255-258): the
    reference's bytes."""
    comp, raw = lz4ada.gen_block(lz4ada.GEN_KINDS["literal"], 0x17, 17 << 20)
    assert len(comp) > 16 << 20
    with pytest.raises(lz4ada.LZ4AdaError):
        run_lone(comp, len(raw))
    # (the buffer holds the whole block: Min_Buffer_Size covers 8 MiB)
    octx = O.Decompressor.init_for_block(len(comp))
    obuf = ctypes.create_string_buffer(len(raw) + 64)
    st, oc, of, ol = octx.update(comp, obuf)
    assert st == O.OK and obuf.raw[of:ol + 1] == raw
    ctx, _ = lz4ada.Decompressor.init_for_block(len(comp))
    buf = bytearray(len(raw) + 64)
    c, f, l = ctx.update(comp, buf)
    assert (c, f, l) == (oc, of, ol)
    assert bytes(buf[f:l + 1]) == raw
