"""Build LZ4 frames (v1.6.3 frame format) from block payloads.

Used by bench.py and the tests to wrap synthetic blocks (lz4ada.gen_block)
into frames with the FLG/BD combinations of BASELINE.json's configs.
Checksums use the `xxhash` package (an implementation independent of both
the product and the oracle).
"""
import struct

import xxhash

MAGIC = 0x184D2204
BD_CODE = {64 << 10: 4, 256 << 10: 5, 1 << 20: 6, 4 << 20: 7}


def header(block_max: int, indep=True, block_cksum=False, content_cksum=False,
           content_size=None) -> bytes:
    flg = 0x40 | (0x20 if indep else 0) | (0x10 if block_cksum else 0) \
        | (0x08 if content_size is not None else 0) | (0x04 if content_cksum else 0)
    bd = BD_CODE[block_max] << 4
    desc = bytes([flg, bd])
    if content_size is not None:
        desc += struct.pack("<Q", content_size)
    hc = (xxhash.xxh32(desc).intdigest() >> 8) & 0xFF
    return struct.pack("<I", MAGIC) + desc + bytes([hc])


def block_record(payload: bytes, stored=False, block_cksum=False) -> bytes:
    word = len(payload) | (0x80000000 if stored else 0)
    rec = struct.pack("<I", word) + payload
    if block_cksum:
        rec += struct.pack("<I", xxhash.xxh32(payload).intdigest())
    return rec


def trailer(content: bytes = None, content_cksum=False, content_hash=None) -> bytes:
    t = struct.pack("<I", 0)
    if content_cksum:
        h = content_hash if content_hash is not None else xxhash.xxh32(content).intdigest()
        t += struct.pack("<I", h)
    return t


def build_frame(blocks, block_max: int, indep=True, block_cksum=False, content_cksum=False,
                with_content_size=False):
    """blocks: list of (payload, decoded, stored) -> (frame bytes, decoded bytes)."""
    decoded = b"".join(b[1] for b in blocks)
    out = [header(block_max, indep, block_cksum, content_cksum,
                  len(decoded) if with_content_size else None)]
    for payload, _, stored in blocks:
        out.append(block_record(payload, stored, block_cksum))
    out.append(trailer(decoded, content_cksum))
    return b"".join(out), decoded
