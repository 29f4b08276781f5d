"""lz4ada_decode_frame_multi (lz4ada_multi.cpp): one frame over n GPUs from
one process, RCCL for the verdict all-reduce and the optional gather.  The
box has one GPU, so n_gpus = 1 (a real one-rank RCCL communicator); the
results must equal the oracle's (oracle/lz4ada_oracle.c, lz4ada.adb) for
clean frames, frames the bulk path rejects and frames that do not shard."""
import pytest

import _oracle as O

import lz4ada
import lz4frame

pytestmark = pytest.mark.gpu

KiB = 1024


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not lz4ada.device_available():
        pytest.fail("MI355X not usable: " + lz4ada._thread_error())


def indep_frame(lens, bmax, seed=3, **kw):
    blocks = [lz4ada.gen_block(i % 4, seed * 100 + i, n) + (False,) for i, n in enumerate(lens)]
    return lz4frame.build_frame(blocks, bmax, indep=True, **kw)


def like_oracle(frame, call):
    st, ref, msg = O.unlz4ada(frame, out_cap=4 * len(frame) + (64 << 20))
    if st == O.OK:
        out, cons = call(frame)
        assert out == ref
        return ref
    with pytest.raises(lz4ada.LZ4AdaError) as ei:
        call(frame)
    assert str(ei.value) == O.exception_information(st, msg)
    return None


@pytest.mark.parametrize("bmax,lens", [
    (4 << 20, [4 << 20] * 6 + [12345]),
    (64 * KiB, [65536] * 40 + [1]),
    (256 * KiB, [262144, 1000, 262144, 5, 262144]),  # short blocks mid-frame: compaction
    (64 * KiB, []),
])
@pytest.mark.parametrize("cks", [(True, True), (False, False), (False, True)])
def test_multi_one_gpu_matches_oracle(bmax, lens, cks):
    frame, raw = indep_frame(lens, bmax, block_cksum=cks[0], content_cksum=cks[1])
    out, cons = lz4ada.decode_frame_multi(frame, 1)
    assert out == raw and cons == len(frame)
    assert lz4ada.last_path() == lz4ada.PATH_INDEPENDENT | lz4ada.PATH_MULTI
    assert like_oracle(frame, lambda f: lz4ada.decode_frame_multi(f, 1, devices=[0])) == raw


def test_multi_content_size_and_trailing_bytes():
    frame, raw = indep_frame([65536] * 5 + [300], 64 * KiB, with_content_size=True,
                             content_cksum=True)
    out, cons = lz4ada.decode_frame_multi(frame + b"trailing", 1)
    assert out == raw and cons == len(frame)


@pytest.mark.parametrize("what", ["block_cksum", "content_cksum", "content_size", "data"])
def test_multi_errors_are_the_references(what):
    lens = [256 * KiB] * 5 + [777]
    blocks = [lz4ada.gen_block(1, 40 + i, n) for i, n in enumerate(lens)]
    raw = b"".join(r for _, r in blocks)
    hdr = lz4frame.header(256 * KiB, indep=True, block_cksum=what != "data", content_cksum=True,
                          content_size=len(raw) + (3 if what == "content_size" else 0))
    recs = [lz4frame.block_record(c, block_cksum=what != "data") for c, _ in blocks]
    if what in ("block_cksum", "data"):
        r = bytearray(recs[3])
        r[60] ^= 0x21
        recs[3] = bytes(r)
    h = lz4frame.xxhash.xxh32(raw).intdigest() ^ (2 if what == "content_cksum" else 0)
    frame = hdr + b"".join(recs) + lz4frame.trailer(content_cksum=True, content_hash=h)
    like_oracle(frame, lambda f: lz4ada.decode_frame_multi(f, 1))
    assert lz4ada.last_path() & lz4ada.PATH_MULTI


def test_multi_linked_and_d2_frames_decode_on_the_first_gpu():
    lb = lz4ada.gen_linked_blocks(1, 9, 256 * KiB, 4)
    for indep in (False, True):  # linked; D2 (B.Indep set, cross-block refs)
        frame, raw = lz4frame.build_frame([(c, r, False) for c, r in lb], 256 * KiB, indep=indep,
                                          block_cksum=True, content_cksum=True)
        assert like_oracle(frame, lambda f: lz4ada.decode_frame_multi(f, 1)) == raw
        assert lz4ada.last_path() & lz4ada.PATH_LINKED


def test_multi_gather_into_device_memory():
    import torch
    frame, raw = indep_frame([1 << 20] * 9 + [4321], 1 << 20, block_cksum=True, content_cksum=True)
    d = torch.zeros(len(raw) + 4096, dtype=torch.uint8, device="cuda:0")
    n, cons = lz4ada.decode_frame_multi_gather(frame, 1, d.data_ptr(), d.numel())
    torch.cuda.synchronize()
    assert n == len(raw) and cons == len(frame)
    assert d[:n].cpu().numpy().tobytes() == raw
    # a linked frame takes the one-GPU path and is copied in
    lb = lz4ada.gen_linked_blocks(1, 4, 256 * KiB, 3)
    lf, lraw = lz4frame.build_frame([(c, r, False) for c, r in lb], 256 * KiB, indep=False)
    n, _ = lz4ada.decode_frame_multi_gather(lf, 1, d.data_ptr(), d.numel())
    torch.cuda.synchronize()
    assert d[:n].cpu().numpy().tobytes() == lraw


def test_multi_device_out_of_range():
    frame, raw = indep_frame([65536] * 2, 64 * KiB)
    import torch
    n = torch.cuda.device_count()
    with pytest.raises(lz4ada.LZ4AdaError, match="out of range"):
        lz4ada.decode_frame_multi(frame, n + 1)


def test_multi_repeated_calls_reuse_workers():
    frame, raw = indep_frame([4 << 20] * 4, 4 << 20, block_cksum=True)
    for _ in range(5):
        assert lz4ada.decode_frame_multi(frame, 1)[0] == raw


def test_multi_repeated_call_allocates_nothing():
    """the worker keeps its device buffers and pinned
    staging across calls -- a repeated call of the same frame makes no new
    device allocation -- and the H2D runs in pinned chunks beside the
    decode (a frame over the 64 MiB staging chunk spans several groups)."""
    frame, raw = indep_frame([4 << 20] * 40 + [777], 4 << 20, block_cksum=True,
                             content_cksum=True)
    out, cons = lz4ada.decode_frame_multi(frame, 1)
    assert out == raw
    n0 = lz4ada.multi_device_allocs(0)
    assert n0 > 0
    for _ in range(2):
        out, cons = lz4ada.decode_frame_multi(frame, 1)
        assert out == raw and cons == len(frame)
    assert lz4ada.multi_device_allocs(0) == n0


def test_rccl_version_reported():
    v = lz4ada.rccl_version()
    assert v >= 20000, v
    print("RCCL bound in this process:", v)
