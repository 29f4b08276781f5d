"""bench.py's launcher (CPU, gloo): `--gpus N` outside a launcher starts N
ranks itself (one process per GPU on the box), the ranks form one process
group of N, and the configs[3] frame (8192 blocks) is split over them."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _run(*argv, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv],
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_launcher_two_ranks():
    r = _run("--gpus", "2", "--launch-check")
    assert r == {"n_gpus": 2, "ranks": 2, "blocks_total": 8192}


def test_launcher_one_rank_no_spawn():
    r = _run("--gpus", "1", "--launch-check")
    assert r == {"n_gpus": 1, "ranks": 1, "blocks_total": 2048}


@pytest.mark.parametrize("world,total", [(2, 8192), (3, 8192), (8, 8192), (8, 100)])
def test_shard_ranges_cover_frame(world, total):
    import bench
    rs = [bench.shard_range(r, world, total) for r in range(world)]
    assert rs[0][0] == 0 and rs[-1][1] == total
    assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
    sizes = [hi - lo for lo, hi in rs]
    assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("first,nblocks,unique", [(0, 10, 4), (3, 10, 4), (5, 3, 8), (0, 64, 64),
                                                  (7, 130, 64)])
def test_assemble_shard_device_tiling(first, nblocks, unique):
    """The shard is one period of unique blocks tiled on the device: bytes
    and descriptors must equal a plain host assembly of the same blocks."""
    import random
    import torch
    import bench
    sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))
    import lz4ada
    rng = random.Random(first * 1000 + nblocks)
    recs = []
    for i in range(unique):
        clen = rng.randrange(5, 300)
        rec = (clen).to_bytes(4, "little") + bytes(rng.randrange(256) for _ in range(clen)) + \
            rng.randrange(1 << 32).to_bytes(4, "little")
        recs.append((rec, clen, 1000 + i, rng.randrange(1 << 32), b"", b""))
    fr, fl, de, eh, cb, rb, descs = bench.assemble_shard(lz4ada, torch, recs, first, nblocks, 4096,
                                                         torch.device("cpu"))
    want = b"".join(recs[(first + i) % unique][0] for i in range(nblocks)) + bytes(64)
    assert fl == len(want) and bytes(fr.numpy().tobytes()) == want
    pos = 0
    for i in range(nblocks):
        r = recs[(first + i) % unique]
        assert descs[i].in_off == pos + 4 and descs[i].in_len == r[1]
        assert descs[i].cksum == int.from_bytes(r[0][4 + r[1]:], "little")
        assert descs[i].flags == lz4ada.BLOCK_HAS_CKSUM
        pos += len(r[0])
    assert eh == [recs[(first + i) % unique][3] for i in range(nblocks)]


def test_kernel_code_hash_guards_traffic_figure():
    """the PMC traffic figure is reused only while the
    headline kernel's machine code is the one it was measured with -- the
    hash is read from the built library's gfx950 code object, per kernel."""
    import bench
    h = bench.kernel_code_hash("k_decode_idx")
    assert h is not None and len(h) == 16
    assert h == bench.kernel_code_hash("k_decode_idx")
    assert h != bench.kernel_code_hash("k_decode_idx_lk")  # not a prefix match
    assert bench.kernel_code_hash("no_such_kernel") is None
    assert bench.kernel_code_hash("k_decode_idx", lib="/nonexistent.so") is None
