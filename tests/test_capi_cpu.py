"""CPU-side checks of the product library (no GPU needed).

* the C-ABI library loads and exports every function include/lz4ada_hip.h
  declares;
* host framing logic (header parser, size-word checks) reproduces the
  reference's exception text for every error vector that fails before any
  block is decoded;
* the frame indexer agrees with an independent walk of the vectors;
* the synthetic block generator emits blocks the oracle decodes to exactly
  the bytes the generator reports;
* decoding without a GPU fails loudly (no CPU fallback).
"""
import ctypes
import os
import re
import struct

import pytest

import _oracle as O
from conftest import ROOT, error_vectors, good_vectors, read_eds, read_vector

import lz4ada
import lz4frame


def header_functions():
    with open(os.path.join(ROOT, "include", "lz4ada_hip.h")) as fh:
        text = fh.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(lz4ada_\w+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    names = header_functions()
    assert len(names) >= 25
    lib = ctypes.CDLL(lz4ada.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(lz4ada.EXPORTED), set(names) ^ set(lz4ada.EXPORTED)
    assert lz4ada._lib.lz4ada_abi_version() == 1


def test_error_names():
    assert lz4ada.error_name(2) == "LZ4ADA.DATA_CORRUPTION"
    assert lz4ada.to_hex(0x184d9904) == "184d9904"
    assert lz4ada.to_hex(0xa7, 8) == "a7"


HEADER_ONLY = ["corruptedmagic", "corruptedhdrchck", "corruptedreserved", "z1ver",
               "corruptedblocksz", "t2e", "cntblkszoverflow"]


@pytest.mark.parametrize("name", HEADER_ONLY)
def test_header_error_vectors_product(name):
    # These fail in Init_With_Header or in the block size word check
    # (lz4ada.adb:541-553), before any block reaches the GPU.
    data = read_vector(name, "err")[:10001]
    try:
        ctx, consumed, mbs = lz4ada.Decompressor.init_with_header(
            data, lz4ada.Reservation.Single_Frame)
        buf = bytearray(mbs)
        total = consumed
        while total < len(data):
            c, f, l = ctx.update(data, buf, total)
            assert c > 0
            total += c
        pytest.fail("no exception")
    except lz4ada.LZ4AdaError as e:
        assert str(e) == read_eds(name)


def test_reservation_exceeded_product():
    tc = read_vector("z2841", "lz4")[:36]
    with pytest.raises(lz4ada.TooLittleMemory):
        lz4ada.Decompressor.init_with_header(tc, lz4ada.Reservation.SZ_64_KiB)


def walk_blocks(data):
    """Independent test-side walk of a single modern frame's size words."""
    flg, bd = data[4], data[5]
    pos = 7 + (8 if flg & 8 else 0) + (4 if flg & 1 else 0)
    out = []
    while True:
        (w,) = struct.unpack_from("<I", data, pos)
        if w == 0:
            break
        n = w & 0x7FFFFFF
        out.append((pos + 4, n, bool(w >> 31)))
        pos += 4 + n + (4 if flg & 16 else 0)
    return out


@pytest.mark.parametrize("name", ["t100k", "t300k", "t301k", "t1111k", "b3444k", "z2841",
                                  "z9m", "z1", "z100", "empty", "t389"])
def test_frame_index_matches_walk(name):
    data = read_vector(name, "lz4")
    info, descs = lz4ada.frame_index(data)
    want = walk_blocks(data)
    assert info.nblocks == len(want)
    for i, (off, n, stored) in enumerate(want):
        d = descs[i]
        assert (d.in_off, d.in_len, bool(d.flags & lz4ada.BLOCK_STORED)) == (off, n, stored)
        assert d.out_off == i * info.block_max
    assert info.independent == (1 if data[4] & 0x20 else 0)


@pytest.mark.parametrize("kind", [0, 1, 2, 3])
@pytest.mark.parametrize("raw_len", [0, 1, 5, 12, 13, 100, 4096, 65536, 300001])
def test_generator_blocks_decode_on_oracle(kind, raw_len):
    comp, raw = lz4ada.gen_block(kind, 1234 + raw_len, raw_len)
    assert len(raw) == raw_len
    bmax = min(b for b in lz4frame.BD_CODE if b >= raw_len)
    frame, decoded = lz4frame.build_frame([(comp, raw, False)], block_max=bmax,
                                          block_cksum=True, content_cksum=True)
    st, out, eof, msg = O.decode_stream(frame)
    assert st == O.OK, msg
    assert out == raw


def test_generator_sequence_density():
    # dense ~5 B/sequence, mixed ~32 B/sequence with ratio ~2
    n = 1 << 20
    comp_d, _ = lz4ada.gen_block(0, 1, n)
    comp_m, _ = lz4ada.gen_block(1, 1, n)
    comp_r, _ = lz4ada.gen_block(2, 1, n)
    assert 0.45 < len(comp_d) / n < 0.9
    assert 0.35 < len(comp_m) / n < 0.65
    assert len(comp_r) / n < 0.01


def test_decode_without_gpu_fails_loudly():
    if lz4ada.device_available():
        pytest.skip("a GPU is present")
    with pytest.raises(lz4ada.DeviceError):
        lz4ada.decode_stream(read_vector("z100", "lz4"))
    ctx, mbs = lz4ada.Decompressor.init()
    buf = bytearray(mbs)
    data = read_vector("z100", "lz4")
    with pytest.raises(lz4ada.DeviceError):
        pos = 0
        while pos < len(data):
            c, f, l = ctx.update(data, buf, pos)
            pos += c


def test_cli_counterparts_built_and_fail_loudly_without_gpu():
    """unlz4ada / xxhash32ada (the reference's CLIs over the C-ABI) exist;
    without a GPU they report the device error instead of decoding on the
    CPU."""
    import subprocess
    from conftest import PKG
    for exe in ("unlz4ada", "xxhash32ada"):
        path = os.path.join(PKG, exe)
        assert os.access(path, os.X_OK), path
    if lz4ada.device_available():
        pytest.skip("a GPU is present (tests/test_gpu_cli.py covers the CLIs)")
    p = subprocess.run([os.path.join(PKG, "unlz4ada")], input=read_vector("z100", "lz4"),
                       capture_output=True, timeout=60)
    assert p.returncode == 1 and p.stdout == b""
    assert p.stderr.decode().startswith("raised LZ4ADA.DEVICE_ERROR : ")


def _hdrinfo_expected(data: bytes) -> str:
    """tool_lz4hdrinfo/lz4hdrinfo.adb:70-145 restated (test side).  The tool
    reads one 64-byte buffer; bytes past a short input (undefined in the
    Ada tool) read as 0 in the counterpart."""
    data = (data + bytes(64))[:64]
    lines = ["Ma_Sys.ma LZ4 Header Info 1.0.0, (c) 2023 Ma_Sys.ma <info@masysma.net>", ""]
    magic = struct.unpack("<I", data[:4])[0]
    tf = lambda b: "TRUE" if b else "FALSE"
    if magic == 0x184D2204:
        flg, bd = data[4], data[5]
        bms = (bd & 0x70) >> 4
        lines += [f"Declared Format        = {magic:08x} (modern)", f"FLG                    = {flg:02x}",
                  f"    Version:64|128     = {(flg & 0xc0) >> 6:02x}",
                  f"    Block_Checksum:16  = {tf(flg & 16)}", f"    Content_Size:8     = {tf(flg & 8)}",
                  f"    Content_Checksum:4 = {tf(flg & 4)}", f"    Reserved:2         = {tf(flg & 2)}",
                  f"    Dictionary_ID:1    = {tf(flg & 1)}", f"BD                     = {bd:02x}",
                  f"    Has_Reserved       = {tf(bd & 0x8f)}",
                  "    Block_Max_Size     = " + {4: "64 KiB", 5: "256 KiB", 6: "1 MiB",
                                                 7: "4 MiB"}.get(bms, "INVALID") + f" ({bms:02x})"]
        cur = 6
        if flg & 8:
            lines.append(f"Content_Size           =  {struct.unpack('<Q', data[cur:cur + 8])[0]}")
            cur += 8
        cur += 4 if flg & 1 else 0
        lines.append(f"Header_Checksum        = {data[cur]:02x}")
    elif magic == 0x184C2102:
        lines.append(f"Declared Format        = {magic:08x} (legacy)")
    elif 0x184D2A50 <= magic <= 0x184D2A5F:
        lines += [f"Declared Format        = {magic:08x} (skippable)",
                  f"Content_Size           =  {struct.unpack('<I', data[4:8])[0]}"]
    else:
        lines.append(f"Declared Format        = {magic:08x} (UNSUPPORTED)")
    return "\n".join(lines) + "\n"


@pytest.mark.parametrize("name", good_vectors() + error_vectors())
def test_lz4hdrinfo(name):
    """The header dumper counterpart (host only, no library) on every vector."""
    import subprocess
    from conftest import PKG
    ext = "lz4" if name in good_vectors() else "err"
    data = read_vector(name, ext)
    p = subprocess.run([os.path.join(PKG, "lz4hdrinfo")], input=data, capture_output=True, timeout=30)
    if len(data) < 7:
        assert p.returncode == 1
        assert p.stderr.decode().startswith("raised CONSTRAINT_ERROR : Partial frame detected.")
    else:
        assert p.returncode == 0
        assert p.stdout.decode() == _hdrinfo_expected(data)


# ------------------------------------------------ XXHash32 over host bytes
# (host chain since round 3: no device needed, so these run on the CPU)

def test_xxh32_kat_byte_feed():
    """lz4test.adb:129-147: 1a x 14, 11, 10 fed one byte at a time."""
    h = lz4ada.XXHash32()
    for b in bytes([0x1a] * 14 + [0x11, 0x10]):
        h.update(bytes([b]))
    assert h.final() == 0xf994ef8a


@pytest.mark.parametrize("n", [0, 1, 3, 15, 16, 17, 31, 32, 33, 1000, 65537])
def test_xxh32_host_matches_oracle_and_xxhash(n):
    import random
    import xxhash
    data = random.Random(n).randbytes(n)
    want = xxhash.xxh32(data).intdigest()
    assert O.xxh32(data) == want
    assert lz4ada.XXHash32.hash(data) == want
    # ragged update sizes continue one chain (Update1 / Process, lz4ada.adb:942-991)
    h = lz4ada.XXHash32(seed=12345)  # Init ignores the seed (quirk Q1)
    pos, step = 0, 1
    while pos < n:
        h.update(data[pos:pos + step])
        pos += step
        step = step * 3 % 37 + 1
    assert h.final() == want


def test_xxh32_reset_honours_seed():
    import xxhash
    h = lz4ada.XXHash32()
    h.reset(7)
    h.update(b"hello world, hello world")
    assert h.final() == xxhash.xxh32(b"hello world, hello world", seed=7).intdigest()
