#!/usr/bin/env python3
"""The C-ABI's host logic under AddressSanitizer, on the CPU (no device):
frame indexing of every reference vector (good, error, truncated at every
length class, bit-flipped), the facade's header / block-framing state machine
up to its first decode (which reports LZ4ADA_DEVICE_ERROR without a GPU), the
host XXH32, shard planning and the block generator.  VERDICT r5 item 7.

    make -C bo-lz4-ada_amd/csrc asan
    LD_PRELOAD=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so) \\
      ASAN_OPTIONS=detect_leaks=0 LZ4ADA_LIB=bo-lz4-ada_amd/liblz4ada_hip_asan.so \\
      python tools/asan_host.py
ASan aborts the process with a report on the first bad access; a clean run
prints the counts."""
import glob
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))
import lz4ada  # noqa: E402
import lz4frame  # noqa: E402

assert "asan" in lz4ada.LIB_PATH, lz4ada.LIB_PATH
frames = []
for p in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "vectors", "*.lz4")) +
                glob.glob(os.path.join(ROOT, "tests", "golden", "lz4f", "*.lz4"))):
    with open(p, "rb") as fh:
        frames.append(fh.read())
for k in (1, 2, 0, 4):
    for kind in (0, 1, 2, 3):
        blocks = lz4ada.gen_linked_blocks(kind, 7 + k, 65536, 3, last_len=1000 * k + 1)
        frames.append(lz4frame.build_frame([(c, r, False) for c, r in blocks], 64 << 10, indep=k % 2 == 0,
                                           block_cksum=k > 1, content_cksum=True)[0])
rng = random.Random(5)
n_idx = n_err = n_upd = 0


def index(data):
    global n_idx, n_err
    try:
        lz4ada.frame_index(data)
        n_idx += 1
    except lz4ada.LZ4AdaError:
        n_err += 1


def facade(data, feed):
    """Init_With_Header + Update at `feed` bytes a call until the first
    decode (a device error here) or an error of the framing itself."""
    global n_upd
    try:
        ctx, pos, mbs = lz4ada.Decompressor.init_with_header(data)
    except lz4ada.LZ4AdaError:
        return
    buf = bytearray(max(mbs, 1))
    for _ in range(64):
        if pos >= len(data):
            break
        try:
            c, f, l = ctx.update(data, buf, pos, min(len(data), pos + feed))
        except lz4ada.LZ4AdaError:
            break
        n_upd += 1
        if c == 0:
            break
        pos += c


for data in frames:
    index(data)
    for cut in sorted({1, 3, 4, 7, 11, 15, 19, len(data) // 2, len(data) - 5, len(data) - 1}):
        if 0 < cut < len(data):
            index(data[:cut])
    for _ in range(40):
        b = bytearray(data)
        for _ in range(rng.randint(1, 4)):
            b[rng.randrange(min(len(b), 64))] ^= 1 << rng.randrange(8)
        index(bytes(b))
    for feed in (1, 7, 4096):
        facade(data[:4096], feed)
        facade(data, feed)
h = lz4ada.XXHash32()
for data in frames:
    h.update(data)
    import xxhash
    assert lz4ada.XXHash32.hash(data[:1000]) == xxhash.xxh32(data[:1000]).intdigest()
info, descs = lz4ada.frame_index(frames[0])
for n in (1, 2, 3, 8):
    lz4ada.plan_shards(descs, info.nblocks, n)
print(f"asan host run clean: {len(frames)} frames, {n_idx} indexed, {n_err} index errors, {n_upd} Update calls",
      flush=True)
