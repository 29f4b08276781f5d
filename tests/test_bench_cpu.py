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
