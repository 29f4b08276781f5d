"""Multi-rank sharding logic on the CPU (gloo, world_size 2).

The GPU decode itself is covered by tests/test_gpu_parity.py; here the
shard plan, the per-rank byte slices and re-based descriptors, and the one
status all-reduce are checked with the oracle standing in as the checker
of each rank's slice (tests only)."""
import ctypes
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import _oracle as O
import lz4ada
import lz4frame
import shard

KiB = 1024


def frame_of(nblocks, block_max=64 * KiB, kinds=(0, 1, 2, 3), short_last=True):
    blocks = []
    for i in range(nblocks):
        raw_len = block_max if (i < nblocks - 1 or not short_last) else block_max // 3 + 7
        comp, raw = lz4ada.gen_block(kinds[i % len(kinds)], 0x4C5A3441 + i, raw_len)
        blocks.append((comp, raw, False))
    return lz4frame.build_frame(blocks, block_max, indep=True, block_cksum=True)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("lens", [[5] * 17, [1, 100, 1, 1, 100, 3], [7], [], [3, 3]])
def test_plan_shards_partition(lens, world):
    plan = shard.plan_shards(lens, world)
    assert len(plan) == world
    assert plan[0][0] == 0 and plan[-1][1] == len(lens)
    for (a, b), (c, d) in zip(plan, plan[1:]):
        assert b == c and a <= b
    if lens and world > 1:
        total, biggest = sum(lens), max(lens)
        for a, b in plan:
            assert sum(lens[a:b]) <= total / world + biggest


def test_plan_shards_balances_uniform_blocks():
    plan = shard.plan_shards([4 << 20] * 8192, 8)
    assert [b - a for a, b in plan] == [1024] * 8


def decode_slice_with_oracle(frame, local, k, b0, b1, out_bytes):
    """What a rank's GPU would hold: every block of its slice at its slot."""
    data = frame[b0:b1]
    out = bytearray(out_bytes)
    lens = []
    for j in range(k):
        d = local[j]
        payload = data[d.in_off:d.in_off + d.in_len]
        if d.flags & lz4ada.BLOCK_HAS_CKSUM:
            assert O.xxh32(payload) == d.cksum
        if d.flags & lz4ada.BLOCK_STORED:
            raw = payload
        else:
            ctx = O.Decompressor.init_for_block(len(payload))
            buf = ctypes.create_string_buffer(ctx.min_buffer_size)
            st, cons, first, last = ctx.update(payload, buf)
            assert st == O.OK and cons == len(payload), ctx.last_error()
            raw = buf.raw[first:last + 1]
        out[d.out_off:d.out_off + len(raw)] = raw
        lens.append(len(raw))
    return out, lens


def _worker(rank, world, port, frame, expected, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        info, descs = lz4ada.frame_index(frame)
        plan = shard.plan_shards([descs[i].in_len for i in range(info.nblocks)], world)
        lo, hi = plan[rank]
        b0, b1, local, out_bytes = shard.shard_slice(descs, lo, hi)
        out, lens = decode_slice_with_oracle(frame, local, hi - lo, b0, b1, out_bytes)
        # one status all-reduce: rank 1 reports an error in the second pass
        ok = shard.reduce_status(shard.SHARD_OK)
        bad = shard.reduce_status(shard.SHARD_BLOCK_ERROR if rank == 1 else shard.SHARD_OK)
        # assemble on rank 0 (test only; the product keeps outputs resident)
        pieces = [None] * world
        dist.all_gather_object(pieces, (lo, hi, bytes(out[:sum(lens)]), lens))
        if rank == 0:
            pieces.sort()
            whole = b"".join(p[2] for p in pieces)
            covered = [i for p in pieces for i in range(p[0], p[1])]
            result_q.put((ok, bad, whole == expected, covered == list(range(info.nblocks)),
                          [p[1] - p[0] for p in pieces]))
    finally:
        dist.destroy_process_group()


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
def test_two_rank_gloo_shards_reassemble_to_the_frame():
    frame, expected = frame_of(9)
    st, out, msg = O.unlz4ada(frame, out_cap=len(expected) + 65536)
    assert st == O.OK and out == expected, msg
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    mp.start_processes(_worker, args=(2, port, frame, expected, q), nprocs=2, join=True,
                       start_method="spawn")
    ok, bad, same, covered, sizes = q.get(timeout=10)
    assert ok == shard.SHARD_OK
    assert bad == shard.SHARD_BLOCK_ERROR
    assert same and covered
    assert all(s > 0 for s in sizes)


def test_linked_frames_do_not_shard():
    blocks = [lz4ada.gen_block(1, 7 + i, 64 * KiB) + (False,) for i in range(2)]
    frame, _ = lz4frame.build_frame(blocks, 64 * KiB, indep=False)
    with pytest.raises(ValueError):
        shard.decode_frame_sharded(frame, 0, 1, torch.device("cpu"))


# ---------------------------------------------- frame-level checks across ranks

class _Info:
    def __init__(self, has_size=False, size=0, cksum=False, declared=0):
        self.has_content_size, self.content_size = has_size, size
        self.content_checksum, self.content_checksum_declared = cksum, declared


def _oracle_hasher(piece):
    """update_local / finalize over the oracle's 48-byte hasher state (the
    checker standing in for the product's D2H + host chain)."""
    L = O.lib()

    def make():
        init = ctypes.create_string_buffer(48)
        L.oracle_xxh32_reset(init, 0)

        def update(state):
            buf = ctypes.create_string_buffer(state, 48)
            L.oracle_xxh32_update(buf, piece, len(piece))
            return buf.raw

        def final(state):
            return L.oracle_xxh32_final(ctypes.create_string_buffer(state, 48))
        return init.raw, update, final
    return make


def _checks_worker(rank, world, port, pieces, infos, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        piece = pieces[rank]
        init, update, final = _oracle_hasher(piece)()
        h = shard.chain_xxh32(init, update, final, rank, world, device="cpu")
        oks = [shard.frame_checks_ok(_Info(*i), len(piece), _oracle_hasher(piece), rank, world,
                                     device="cpu") for i in infos]
        result_q.put((rank, h, oks))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [1, 2, 3])
def test_content_checksum_chains_across_ranks(world):
    """chain_xxh32 = XXH32 of the concatenation in rank order, on every rank
    (empty shares included), and frame_checks_ok agrees with the declared
    content size / checksum exactly as Check_End_Mark would."""
    import random
    import xxhash
    rng = random.Random(world)
    sizes = [rng.randint(0, 70000) for _ in range(world)]
    if world > 1:
        sizes[1] = 0  # a rank with no blocks passes the state on unchanged
    pieces = [rng.randbytes(n) for n in sizes]
    whole = b"".join(pieces)
    want = xxhash.xxh32(whole).intdigest()
    infos = [(False, 0, False, 0), (True, len(whole), True, want), (True, len(whole) + 1, False, 0),
             (False, 0, True, want ^ 1), (True, len(whole), False, 0)]
    expect = [True, True, False, False, True]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_checks_worker, args=(world, free_port(), pieces, infos, q), nprocs=world,
                       join=True, start_method="spawn")
    res = sorted(q.get(timeout=10) for _ in range(world))
    for rank, h, oks in res:
        assert h == want, rank
        assert oks == expect, rank


def test_empty_frame_chain_hash():
    init, update, final = _oracle_hasher(b"")()
    assert shard.chain_xxh32(init, update, final, 0, 1) == shard.XXH32_EMPTY
