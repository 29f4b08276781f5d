"""Sharded decode on the GPU with a real process group: world
1-3 ranks on the one GPU of the box, gloo for the collectives (coll_device
"cpu"), every rank decoding its share through the C-ABI.  Frame-level checks
(declared content size, content checksum chained in frame order) and the
error paths must give what the reference gives for the whole frame
(lz4ada.adb:463-523, 661-707): the oracle's exception text, on every rank.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp

import _oracle as O

import lz4ada
import lz4frame

pytestmark = pytest.mark.gpu

KiB = 1024


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, frame, q):
    import torch
    import torch.distributed as dist
    import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        try:
            d_out, (lo, hi), lens = shard.decode_frame_sharded(
                frame, rank, world, torch.device("cuda", 0), coll_device="cpu")
            host = d_out.cpu().numpy().tobytes()
            info, descs = lz4ada.frame_index(frame)
            base = descs[lo].out_off if hi > lo else 0
            got = b"".join(host[descs[lo + j].out_off - base:descs[lo + j].out_off - base + n]
                           for j, n in enumerate(lens))
            # a digest, not the bytes: a child blocks at exit until a large
            # queued item has been read
            q.put((rank, "ok", (len(got), lz4frame.xxhash.xxh32(got).intdigest())))
        except lz4ada.LZ4AdaError as e:
            q.put((rank, "err", str(e)))
        except ValueError as e:
            q.put((rank, "value", str(e)))
    finally:
        dist.destroy_process_group()


def run_world(frame, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pc = mp.start_processes(_worker, args=(world, free_port(), frame, q), nprocs=world,
                            join=False, start_method="spawn")
    res = sorted(q.get(timeout=120) for _ in range(world))
    while not pc.join(timeout=60):
        pass
    return res


def frame_with(what):
    blocks = []
    for i in range(7):
        n = 256 * KiB if i < 6 else 1000
        comp, raw = lz4ada.gen_block(i % 4, 300 + i, n)
        blocks.append((comp, raw, False))
    raw = b"".join(r for _, r, _ in blocks)
    if what == "d2":
        lb = lz4ada.gen_linked_blocks(1, 9, 256 * KiB, 4)
        blocks = [(c, r, False) for c, r in lb]
        raw = b"".join(r for _, r, _ in blocks)
    size = len(raw) + (5 if what == "content_size" else 0)
    hdr = lz4frame.header(256 * KiB, indep=True, block_cksum=True, content_cksum=True,
                          content_size=size)
    recs = [lz4frame.block_record(c, block_cksum=True) for c, _, _ in blocks]
    if what == "block_cksum":
        r = bytearray(recs[4])
        r[200] ^= 0x40
        recs[4] = bytes(r)
    h = lz4frame.xxhash.xxh32(raw).intdigest() ^ (0x100 if what == "content_cksum" else 0)
    return hdr + b"".join(recs) + lz4frame.trailer(content_cksum=True, content_hash=h), raw


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [1, 2, 3])
@pytest.mark.parametrize("what", ["clean", "block_cksum", "content_cksum", "content_size", "d2"])
def test_sharded_frame_checks(what, world):
    frame, raw = frame_with(what)
    st, ref, msg = O.unlz4ada(frame, out_cap=len(raw) + (1 << 20))
    res = run_world(frame, world)
    if what == "clean":
        assert st == O.OK and ref == raw, msg
        assert [r[1] for r in res] == ["ok"] * world
        # every rank's share, in rank order, is the frame's output
        pos = 0
        for _, _, (n, h) in res:
            assert lz4frame.xxhash.xxh32(raw[pos:pos + n]).intdigest() == h
            pos += n
        assert pos == len(raw)
    elif what == "d2":
        # B.Indep set, blocks read earlier blocks: the reference decodes it
        # (linked); it does not shard, rank 0 returns it whole
        assert st == O.OK and ref == raw, msg
        assert [r[1] for r in res] == ["ok"] * world
        n, h = res[0][2]
        assert n == len(raw) and h == lz4frame.xxhash.xxh32(raw).intdigest()
        assert all(r[2][0] == 0 for r in res[1:])
    else:
        assert st != O.OK
        want = O.exception_information(st, msg)
        assert [(r[1], r[2]) for r in res] == [("err", want)] * world
