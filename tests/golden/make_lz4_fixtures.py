#!/usr/bin/env python3
"""Encoder-independent LZ4 frame fixtures.

Run in the build container only:
    python tests/golden/make_lz4_fixtures.py

Every other synthetic frame in the test suite comes from the product's own
generator (csrc/lz4gen.cpp).  These frames come from an independent encoder:
the container's system liblz4 (liblz4.so.1, v1.9.3, the reference LZ4 frame
library), driven through ctypes with LZ4F_compressFrame.  The inputs are
deterministic (seeded) pseudo-text and random bytes; nothing here reads
/root/reference.

For each frame the table records the input's digest and the oracle's
result (oracle/lz4ada_oracle.c, the C restatement of lib/lz4ada.adb): for
the ordinary frames the oracle's output must BE the encoder's input (that
pins the oracle against liblz4 itself); for the quirk-D1 frames it is the
reference's corrupted output (lib/lz4ada.adb:811-817,
862-879), recorded as the oracle gives it.

Frames (tests/golden/lz4f/*.lz4, digests in tests/golden/lz4f_digests.json):
  linked64k      LZ4F defaults: 64 KiB linked blocks, content checksum, level 1
  linked256k     256 KiB linked blocks, block + content checksum, level 9 (HC)
  indep64k       64 KiB independent blocks, block checksum, level 1
  indep4m        4 MiB independent blocks, content size + content checksum
  mix64k         64 KiB independent blocks alternating random (stored) and text
  d1_l13_o65529  64 KiB linked: a stored 64 KiB block, then L literals and a
  d1_l3_o65533   match >= 65,529 back (quirk D1), level 12; no content
  d1_l20_o65535  checksum, so the output is the reference's corrupted bytes
  d1_l1_o65535   (l13_o65529 reads none of the overshoot: output == input)
  d1_cksum       the same shape with a content checksum: the reference raises
  big4m          8 MiB of text in 4 MiB independent blocks, block checksums:
                 tiled TILE times by the GPU tests and bench.py (independent
                 blocks repeat freely) -- the bulk decoder's 2,048-block shape
  big256k        8 MiB of text in 256 KiB linked blocks, block checksums: its
                 32 blocks tiled TILE times (the first block reads no history,
                 so every copy decodes as the first did) -- 4,096 linked blocks

Each entry also lists the XXH32 of every block's decoded bytes
("block_xxh32": the input's block-sized slices, for frames whose output is
their input), and the tiled frames the XXH32 of their whole tiled output.
"""
import ctypes
import hashlib
import json
import os
import random
import sys

import xxhash

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "lz4f")
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))

LIBLZ4 = "liblz4.so.1"
KiB, MiB = 1 << 10, 1 << 20


class FrameInfo(ctypes.Structure):  # LZ4F_frameInfo_t (lz4frame.h, v1.9.x)
    _fields_ = [("blockSizeID", ctypes.c_int), ("blockMode", ctypes.c_int),
                ("contentChecksumFlag", ctypes.c_int), ("frameType", ctypes.c_int),
                ("contentSize", ctypes.c_ulonglong), ("dictID", ctypes.c_uint),
                ("blockChecksumFlag", ctypes.c_int)]


class Prefs(ctypes.Structure):  # LZ4F_preferences_t
    _fields_ = [("frameInfo", FrameInfo), ("compressionLevel", ctypes.c_int),
                ("autoFlush", ctypes.c_uint), ("favorDecSpeed", ctypes.c_uint),
                ("reserved", ctypes.c_uint * 3)]


BSIZE = {64 * KiB: 4, 256 * KiB: 5, 1 * MiB: 6, 4 * MiB: 7}


def lz4f():
    lib = ctypes.CDLL(LIBLZ4)
    lib.LZ4F_compressFrameBound.restype = ctypes.c_size_t
    lib.LZ4F_compressFrameBound.argtypes = [ctypes.c_size_t, ctypes.POINTER(Prefs)]
    lib.LZ4F_compressFrame.restype = ctypes.c_size_t
    lib.LZ4F_compressFrame.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p,
                                       ctypes.c_size_t, ctypes.POINTER(Prefs)]
    lib.LZ4F_isError.restype = ctypes.c_uint
    lib.LZ4F_isError.argtypes = [ctypes.c_size_t]
    lib.LZ4_versionString.restype = ctypes.c_char_p
    return lib


def compress(lib, data, block, linked, level=1, bcksum=False, ccksum=False, csize=False):
    p = Prefs()
    p.frameInfo.blockSizeID = BSIZE[block]
    p.frameInfo.blockMode = 0 if linked else 1
    p.frameInfo.contentChecksumFlag = 1 if ccksum else 0
    p.frameInfo.blockChecksumFlag = 1 if bcksum else 0
    p.frameInfo.contentSize = len(data) if csize else 0
    p.compressionLevel = level
    cap = lib.LZ4F_compressFrameBound(len(data), ctypes.byref(p))
    dst = ctypes.create_string_buffer(cap)
    n = lib.LZ4F_compressFrame(dst, cap, data, len(data), ctypes.byref(p))
    assert not lib.LZ4F_isError(n), "LZ4F_compressFrame failed"
    return dst.raw[:n]


def text(seed, n):
    """Deterministic pseudo-text (Zipf-distributed words): LZ4 ratio ~3."""
    r = random.Random(seed)
    letters = "etaoinshrdlucmfwypvbgkjqxz"
    vocab = ["".join(r.choice(letters) for _ in range(r.randint(2, 9))) for _ in range(400)]
    weights = [1.0 / (k + 1) for k in range(len(vocab))]
    out, size = [], 0
    while size < n:
        words = r.choices(vocab, weights, k=4096)
        chunk = (" ".join(words) + ".\n").encode()
        out.append(chunk)
        size += len(chunk)
    return b"".join(out)[:n]


def d1_input(seed, lit_len, off):
    """A 64 KiB random block (stored by the encoder), then lit_len random
    literals and a 32-byte marker that occurred once in the first block, at
    the position that makes the match exactly `off` back, then random tail."""
    r = random.Random(seed)
    marker = bytes(r.getrandbits(8) for _ in range(32))
    pos2 = 64 * KiB + lit_len  # the marker's second occurrence
    pos1 = pos2 - off
    assert 0 <= pos1 and pos1 + 32 <= 64 * KiB
    b1 = bytearray(r.getrandbits(8) for _ in range(64 * KiB))
    b1[pos1:pos1 + 32] = marker
    b2 = bytes(r.getrandbits(8) for _ in range(lit_len)) + marker + \
        bytes(r.getrandbits(8) for _ in range(600))
    return bytes(b1) + b2


# copies of the big frames' block sequences in the tiled frames
TILE = {"big4m": 128, "big256k": 128}


def digest(b):
    return {"len": len(b), "sha256": hashlib.sha256(b).hexdigest(), "xxh32": xxhash.xxh32(b).intdigest()}


def main():
    import _oracle as O
    lib = lz4f()
    os.makedirs(OUT, exist_ok=True)
    specs = {
        "linked64k": (text(1, 1 * MiB + 12345), dict(block=64 * KiB, linked=True, ccksum=True)),
        "linked256k": (text(2, 1536 * KiB + 777), dict(block=256 * KiB, linked=True, level=9,
                                                       bcksum=True, ccksum=True)),
        "indep64k": (text(3, 1 * MiB + 99), dict(block=64 * KiB, linked=False, bcksum=True)),
        "indep4m": (text(4, 4 * MiB + 654321), dict(block=4 * MiB, linked=False, ccksum=True,
                                                  csize=True)),
        "mix64k": (b"".join((random.Random(50 + i).randbytes(64 * KiB) if i % 2 else text(60 + i, 64 * KiB))
                            for i in range(12)) + text(99, 5000),
                   dict(block=64 * KiB, linked=False, bcksum=True)),
        "d1_l13_o65529": (d1_input(7, 13, 65529), dict(block=64 * KiB, linked=True, level=12)),
        "d1_l3_o65533": (d1_input(8, 3, 65533), dict(block=64 * KiB, linked=True, level=12)),
        "d1_l20_o65535": (d1_input(9, 20, 65535), dict(block=64 * KiB, linked=True, level=12)),
        "d1_l1_o65535": (d1_input(11, 1, 65535), dict(block=64 * KiB, linked=True, level=12)),
        "d1_cksum": (d1_input(10, 1, 65534), dict(block=64 * KiB, linked=True, level=12, ccksum=True)),
        "big4m": (text(5, 8 * MiB), dict(block=4 * MiB, linked=False, bcksum=True)),
        "big256k": (text(6, 8 * MiB), dict(block=256 * KiB, linked=True, bcksum=True)),
    }
    table = {"encoder": "liblz4 " + lib.LZ4_versionString().decode() + " (LZ4F_compressFrame, ctypes)",
             "frames": {}}
    for name, (data, kw) in specs.items():
        frame = compress(lib, data, **kw)
        with open(os.path.join(OUT, name + ".lz4"), "wb") as fh:
            fh.write(frame)
        st, out, _, msg = O.decode_stream(frame)
        ent = {"input": digest(data), "params": {k: v for k, v in kw.items()},
               "frame_len": len(frame), "oracle_status": st,
               "oracle_output": digest(out) if st == O.OK else None,
               "oracle_error": None if st == O.OK else O.exception_information(st, msg)}
        ent["output_is_input"] = st == O.OK and out == data
        if ent["output_is_input"]:
            blk = kw["block"]
            ent["block_xxh32"] = [xxhash.xxh32(data[i:i + blk]).intdigest() for i in range(0, len(data), blk)]
        if name in TILE:
            h = xxhash.xxh32()
            for _ in range(TILE[name]):
                h.update(data)
            ent["tile"] = {"copies": TILE[name], "output_len": TILE[name] * len(data),
                           "output_xxh32": h.intdigest()}
        table["frames"][name] = ent
        print(f"{name}: {len(data)} -> {len(frame)} bytes, oracle status {st}, "
              f"output == input: {ent['output_is_input']}")
    with open(os.path.join(HERE, "lz4f_digests.json"), "w") as fh:
        json.dump(table, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
