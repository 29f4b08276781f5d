"""The multi-GPU C-ABI entry (lz4ada_multi.cpp) without a GPU: its block
planner against shard.py's (one rule for both multi-GPU paths), and the
argument checks that come before any device call."""
import ctypes
import random

import pytest

import lz4ada
import shard


def descs_of(lens):
    d = (lz4ada.BlockDesc * max(len(lens), 1))()
    off = 0
    for i, n in enumerate(lens):
        d[i].in_off, d[i].in_len = off, n
        off += n + 4
    return d


@pytest.mark.parametrize("seed", range(40))
def test_plan_matches_shard_py(seed):
    rng = random.Random(seed)
    nb = rng.choice([0, 1, 2, 3, 7, 64, 500])
    lens = [rng.choice([0, 1, 17, 4096, 65536, 4 << 20, rng.randrange(1, 5 << 20)])
            for _ in range(nb)]
    for n in (1, 2, 3, 5, 8, 13):
        got = lz4ada.plan_shards(descs_of(lens), nb, n)
        assert got == shard.plan_shards(lens, n)
        assert got[0][0] == 0 and got[-1][1] == nb
        assert all(a[1] == b[0] for a, b in zip(got, got[1:]))


def test_plan_configs3_even_split():
    # BASELINE configs[3]: 8192 equal 4 MiB blocks over 8 GPUs -> 1024 each
    lens = [2 << 20] * 8192
    got = lz4ada.plan_shards(descs_of(lens), 8192, 8)
    assert got == [(1024 * r, 1024 * (r + 1)) for r in range(8)]


def test_plan_rejects_bad_arguments():
    with pytest.raises(lz4ada.LZ4AdaError):
        lz4ada.plan_shards(descs_of([5]), 1, 0)


def test_multi_rejects_zero_gpus():
    out = bytearray(16)
    olen, cons = ctypes.c_int64(), ctypes.c_int64()
    st = lz4ada._lib.lz4ada_decode_frame_multi(lz4ada._addr(b"\x04\x22\x4d\x18"), 4, 0, None,
                                               lz4ada._addr(out), 16, ctypes.byref(olen),
                                               ctypes.byref(cons))
    assert st == 6  # LZ4ADA_ASSERTION_ERROR (Pre violated)


def test_multi_without_gpu_is_a_device_error():
    if lz4ada.device_available():
        pytest.skip("a GPU is present")
    out = bytearray(16)
    olen, cons = ctypes.c_int64(), ctypes.c_int64()
    st = lz4ada._lib.lz4ada_decode_frame_multi(lz4ada._addr(b"\x04\x22\x4d\x18"), 4, 1, None,
                                               lz4ada._addr(out), 16, ctypes.byref(olen),
                                               ctypes.byref(cons))
    assert st == 8  # LZ4ADA_DEVICE_ERROR: no CPU fallback
