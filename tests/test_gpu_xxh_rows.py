"""Per-block XXH32 kernel (k_xxh32_rows, four blocks per wave) against the
oracle's XXHash32.Hash (lz4ada.adb:979-1017 restated in oracle/): ragged
lengths (0..15 bytes, exact stripes, one over), every start alignment, a
block count that leaves the last wave's rows partly empty, blocks without
B.Checksum (left untouched), and both entry points -- block checksums over
the frame bytes and output hashes over decoded slots."""
import random

import pytest

import _oracle as O
import lz4ada

pytestmark = pytest.mark.gpu

LENS = [0, 1, 3, 4, 15, 16, 17, 31, 32, 63, 64, 65, 255, 256, 257, 1023, 1024, 1025, 4095,
        4096, 4097, 65535, 65536, 65537, 300001]


def _case(seed, nblocks):
    rnd = random.Random(seed)
    buf = bytes(rnd.getrandbits(8) for _ in range(1 << 20))
    descs = (lz4ada.BlockDesc * nblocks)()
    for i in range(nblocks):
        n = LENS[i % len(LENS)] if i < 2 * len(LENS) else rnd.randrange(0, 200000)
        off = rnd.randrange(0, len(buf) - n + 1)
        descs[i].in_off = off
        descs[i].in_len = n
        descs[i].out_off = off
        descs[i].out_cap = n
        descs[i].flags = 0 if i % 7 == 5 else lz4ada.BLOCK_HAS_CKSUM
    return buf, descs


@pytest.mark.parametrize("nblocks", [1, 3, 4, 5, 37, 64, 129])
def test_block_checksums_rows(nblocks):
    torch = pytest.importorskip("torch")
    buf, descs = _case(1000 + nblocks, nblocks)
    dev = torch.device("cuda:0")
    d_buf = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(dev)
    d_desc = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(dev)
    sentinel = 0x5A5A5A5A
    st = (lz4ada.BlockStatus * nblocks)()
    for s in st:
        s.cksum = sentinel
    d_st = torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8).to(dev)
    sh = torch.cuda.current_stream().cuda_stream
    lz4ada.launch_block_checksums(d_buf.data_ptr(), d_desc.data_ptr(), nblocks, d_st.data_ptr(), sh)
    torch.cuda.synchronize()
    got = (lz4ada.BlockStatus * nblocks).from_buffer_copy(d_st.cpu().numpy().tobytes())
    for i, d in enumerate(descs):
        if d.flags & lz4ada.BLOCK_HAS_CKSUM:
            want = O.xxh32(buf[d.in_off:d.in_off + d.in_len])
            assert got[i].cksum == want, (i, d.in_off, d.in_len)
        else:
            assert got[i].cksum == sentinel, i


@pytest.mark.parametrize("nblocks", [2, 6, 41])
def test_output_hashes_rows(nblocks):
    torch = pytest.importorskip("torch")
    buf, descs = _case(2000 + nblocks, nblocks)
    dev = torch.device("cuda:0")
    d_buf = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(dev)
    d_desc = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(dev)
    st = (lz4ada.BlockStatus * nblocks)()
    for i, d in enumerate(descs):
        st[i].out_len = d.in_len
    d_st = torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8).to(dev)
    d_hash = torch.zeros(nblocks, dtype=torch.int32, device=dev)
    sh = torch.cuda.current_stream().cuda_stream
    lz4ada.output_checksums_device(d_buf.data_ptr(), d_desc.data_ptr(), d_st.data_ptr(), nblocks,
                                   d_hash.data_ptr(), sh)
    torch.cuda.synchronize()
    got = [h & 0xffffffff for h in d_hash.cpu().tolist()]
    for i, d in enumerate(descs):
        assert got[i] == O.xxh32(buf[d.out_off:d.out_off + d.in_len]), (i, d.out_off, d.in_len)
