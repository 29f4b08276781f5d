"""The bulk decoders at their production launch shapes on encoder-produced
data: the liblz4 1.9.3 frames big4m (4 MiB independent
blocks) and big256k (256 KiB linked blocks) of tests/golden/lz4f/, made by
tests/golden/make_lz4_fixtures.py, tiled on the host to 2,048 / 1,024 blocks
and to 4,096 linked blocks.  Golden values are the encoder input's digests
recorded in tests/golden/lz4f_digests.json -- nothing here comes from the
repo's generator (csrc/lz4gen.cpp) or from the decoder under test.

Tiling is valid LZ4: independent blocks repeat freely, and the linked frame's
first block reads no history, so every copy of the 32-block sequence decodes
as the first one does (the reference's round state -- Output_Pos,
Output_Pos_History, lib/lz4ada.adb:678-690 -- is the same at each copy's
start: every 256 KiB block is a round of its own)."""
import json
import os
import struct

import pytest
import xxhash

from conftest import GOLDEN

import bench
import lz4ada
import lz4frame

pytestmark = pytest.mark.gpu

TABLE = json.load(open(os.path.join(GOLDEN, "lz4f_digests.json")))["frames"]
MiB = 1 << 20


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not lz4ada.device_available():
        pytest.fail("MI355X not usable: " + lz4ada._thread_error())


def big4m_recs():
    ent = TABLE["big4m"]
    n = ent["input"]["len"]
    lens = [min(4 * MiB, n - i) for i in range(0, n, 4 * MiB)]
    return bench.golden_recs(lz4ada, os.path.join(GOLDEN, "lz4f", "big4m.lz4"), ent["block_xxh32"], lens)


@pytest.mark.parametrize("nblocks,kernel", [(2048, "k_decode_idx"), (1024, "k_decode_pp2")])
def test_big4m_tiled_bulk(nblocks, kernel):
    """lz4ada_decode_blocks_device (block checksums beside the index decoder)
    on nblocks liblz4 blocks: k_decode_idx's 2,048-block launch and
    k_decode_pp2's at most one block per SIMD; every block OK, its checksum
    and its decoded XXH32 the encoder's."""
    import torch
    assert lz4ada.bulk_decoder_kernel(nblocks) == kernel
    dev = torch.device("cuda", 0)
    recs = big4m_recs()
    fr, fl, de, eh, cb, rb, descs = bench.assemble_shard(lz4ada, torch, recs, 0, nblocks, 4 * MiB, dev)
    assert rb == nblocks * 4 * MiB
    d_out = torch.empty(nblocks * 4 * MiB, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(nblocks * 32, dtype=torch.uint8, device=dev)
    d_hash = torch.zeros(nblocks, dtype=torch.int32, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    lz4ada.decode_blocks_device(fr.data_ptr(), fl, de.data_ptr(), nblocks, d_out.data_ptr(),
                                d_st.data_ptr(), sh)
    torch.cuda.synchronize()
    st = bench.golden_check(lz4ada, torch, d_st, descs, nblocks, d_out.data_ptr(), de.data_ptr(),
                            d_st.data_ptr(), d_hash, eh, sh, "big4m")
    assert sum(s.out_len for s in st) == rb


def tiled_linked_frame(name, copies):
    """The frame's header and its block records `copies` times, then the end
    mark (no content checksum: the header's FLG has none)."""
    with open(os.path.join(GOLDEN, "lz4f", name + ".lz4"), "rb") as fh:
        data = fh.read()
    info, descs = lz4ada.frame_index(data)
    flg = data[4]
    assert not (flg & 0x20) and not (flg & 0x04) and not (flg & 0x08)  # linked, no content cksum / size
    ck = 4 if flg & 0x10 else 0
    first = descs[0].in_off - 4
    last = descs[info.nblocks - 1].in_off + descs[info.nblocks - 1].in_len + ck
    return data[:first] + data[first:last] * copies + struct.pack("<I", 0), info.nblocks * copies


def test_big256k_tiled_linked():
    """4,096 linked 256 KiB liblz4 blocks through lz4ada_decode_frame (the
    linked bulk path: every block against synthetic history, resolved on the
    GPU): the whole output's XXH32 and length are the tiled input's, and no
    block needed the reference-exact path."""
    tile = TABLE["big256k"]["tile"]
    frame, nblocks = tiled_linked_frame("big256k", tile["copies"])
    assert nblocks == 4096
    out, used = lz4ada.decode_frame(frame)
    assert used == len(frame)
    assert len(out) == tile["output_len"]
    assert xxhash.xxh32(out).intdigest() == tile["output_xxh32"]
    path = lz4ada.last_path()
    assert path & lz4ada.PATH_LINKED and not path & lz4ada.PATH_EXACT, path
