#!/usr/bin/env python3
"""bench.py -- MI355X LZ4Ada decode throughput (BASELINE.json metric).

One step = the hot path over one batch: every block of this rank's shard of
a synthetic 4 MiB-block independent frame goes through the GPU block
checksum (XXH32 of each compressed payload, lz4ada.adb:698-707) and the
GPU block decoder (lz4ada.adb:716-904), input already resident in HBM,
output left in HBM.

Workloads (config.workload):
* N = 1 (the default): 2048 x 4 MiB blocks = 8 GiB decoded, FLG 0x70
  (version 01 | B.Indep | B.Checksum), BD 0x70 -- configs[2]'s size, the
  HBM roofline run.  The content-checksum variant (configs[2], FLG 0x74) is
  reported separately as `e2e_content_checksum`: a frame-wide XXH32 is one
  serial chain.
* N > 1: configs[3] itself -- a 32 GiB frame (8192 x 4 MiB blocks, FLG
  0x70) split into N contiguous block ranges, one per rank (strong
  scaling); `value` is the whole frame's decoded bytes / max-over-ranks
  time.  `--gpus N` starts the N ranks itself (torch.distributed.run, one
  process per GPU, RCCL) unless it already runs under a launcher.

Synthetic data: 64 unique blocks from the repo's deterministic LZ4
sequence generator (seed 0x4C5A3441 + i), tiled to size; each rank's shard
is assembled in host memory and copied to the GPU once.  Golden check:
per-block XXH32 of every decoded slot (on the GPU) against the generator's
plaintext hash, after the warmup.

Multi-GPU: one process per GPU (torch.distributed, RCCL); blocks shard
across ranks with no data-path collective.  Timing: barrier +
synchronize on both sides of exactly K steps, max over ranks.  The one
status all-reduce (MAX) runs after the timed region.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))

METRIC = "decompressed MiB/s + achieved HBM GB/s vs roofline, 4MiB-block frame @1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SEED0 = 0x4C5A3441
MiB = 1 << 20
C3_BLOCKS = 8192  # configs[3]: 32 GiB of 4 MiB blocks


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--kind", default="mixed")
    ap.add_argument("--blocks", type=int, default=0,
                    help="blocks of the whole frame (default: 2048 at N=1, configs[3]'s 8192 "
                         "split over the ranks at N>1)")
    ap.add_argument("--block-max", type=int, default=4 * MiB)
    ap.add_argument("--unique", type=int, default=64)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--classes", default="stored,literal,dense,rle",
                    help="extra content classes timed through the product call (N=1 only)")
    ap.add_argument("--real", default="t1111k,liblz4_text",
                    help="encoder-produced classes timed through the product call (N=1 only)")
    ap.add_argument("--no-linked", action="store_true",
                    help="skip the configs[4] row (1 GiB linked frame, 256 KiB blocks)")
    ap.add_argument("--no-64k", action="store_true",
                    help="skip the configs[1] row (1 GiB frame, 64 KiB blocks)")
    ap.add_argument("--no-c3", action="store_true",
                    help="skip the c3_one_gpu row (configs[3]'s 32 GiB frame on one GPU)")
    ap.add_argument("--no-facade", action="store_true",
                    help="skip the facade row (Update at 4 KiB reads from C, SURVEY §8f item 1)")
    ap.add_argument("--launch-check", action="store_true",
                    help="test hook: start the ranks, check the process group (gloo, no GPU), "
                         "print one JSON line")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_decode.json"))
    return ap.parse_args(argv)


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """--gpus N outside a launcher: start N ranks with torch.distributed.run
    (one process per GPU) as a child and return its exit code.  Runs before
    anything touches the GPU in this process."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def kernel_code_hash(kernel: str = "k_decode_idx", lib: str = None) -> str:
    """sha256 (16 hex digits) of one kernel's gfx950 machine code and kernel
    descriptor, read from the built library (the clang offload bundles in
    liblz4ada_hip.so, the code object's symbol table): profiles/pmc_decode.json
    records the hash it was measured with, and bench.py reports its traffic
    only while the hash still matches -- a change to that kernel's code or
    resources voids the figure, a change elsewhere does not (the descriptor's
    code-entry offset, which moves when other kernels are added, is left
    out).  None when the
    library or the kernel is not found."""
    import hashlib
    import struct
    lib = lib or os.environ.get("LZ4ADA_LIB") or os.path.join(ROOT, "bo-lz4-ada_amd", "liblz4ada_hip.so")
    try:
        with open(lib, "rb") as fh:
            d = fh.read()
    except OSError:
        return None
    want = f"{len(kernel)}{kernel}E"  # the mangled name's identifier (not its longer relatives)
    i = 0
    while True:
        i = d.find(b"__CLANG_OFFLOAD_BUNDLE__", i)
        if i < 0:
            return None
        n, p = struct.unpack_from("<Q", d, i + 24)[0], i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", d, p)
            trip = d[p + 24:p + 24 + tl].decode(errors="replace")
            p += 24 + tl
            if "gfx950" not in trip or not size:
                continue
            elf = d[i + off:i + off + size]
            shoff, = struct.unpack_from("<Q", elf, 0x28)
            shentsize, shnum = struct.unpack_from("<HH", elf, 0x3a)
            secs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + k * shentsize) for k in range(shnum)]
            parts = {}
            for sym in (s for s in secs if s[1] == 2):  # SHT_SYMTAB
                strtab = secs[sym[6]]
                for k in range(sym[5] // 24):
                    nm, info, _, shndx, val, sz = struct.unpack_from("<IBBHQQ", elf, sym[4] + 24 * k)
                    name = elf[strtab[4] + nm:elf.index(b"\0", strtab[4] + nm)].decode(errors="replace")
                    if want in name and 0 < shndx < len(secs) and sz:
                        sec = secs[shndx]
                        part = bytearray(elf[sec[4] + val - sec[3]:sec[4] + val - sec[3] + sz])
                        if name.endswith(".kd") and len(part) >= 24:
                            part[16:24] = bytes(8)  # kernel_code_entry_byte_offset: where the code lies
                        parts[name] = bytes(part)
            if parts:
                h = hashlib.sha256()
                for name in sorted(parts):
                    h.update(name.encode())
                    h.update(parts[name])
                return h.hexdigest()[:16]
        i += 24


# ------------------------------------------------------------- synthetic data

def make_unique_blocks(lz4ada, lz4frame, xxhash, kind, n_unique, block_max, block_cksum=True):
    """-> list of (record bytes incl. size word [+ checksum], payload len,
    raw len, raw xxh32, payload, raw).  kind "stored": random bytes in
    uncompressed blocks (size word bit 31, lz4ada.adb:536-538, 686-694)."""
    import numpy as np
    recs = []
    for i in range(n_unique):
        if kind == "stored":
            raw = np.random.default_rng(SEED0 + i).integers(0, 256, block_max, dtype=np.uint8)
            comp = raw = raw.tobytes()
            rec = lz4frame.block_record(comp, stored=True, block_cksum=block_cksum)
        else:
            comp, raw = lz4ada.gen_block(lz4ada.GEN_KINDS[kind], SEED0 + i, block_max)
            rec = lz4frame.block_record(comp, stored=False, block_cksum=block_cksum)
        recs.append((rec, len(comp), len(raw), xxhash.xxh32(raw).intdigest(), comp, raw))
    return recs


def assemble_shard(lz4ada, torch, recs, first_block, nblocks, block_max, dev, slot_pad=0):
    """This rank's shard of the tiled frame: the unique blocks cycle with
    period len(recs) from `first_block`, so one period (rotated to start
    there) is assembled in host memory, copied to the GPU once and tiled on
    the device -- a 16 GiB shard costs one ~130 MiB host assembly."""
    import numpy as np
    n_unique = len(recs)
    period = min(n_unique, nblocks)
    order = [(first_block + i) % n_unique for i in range(period)]
    lens = [len(recs[u][0]) for u in order]
    poffs, pos = [], 0
    for ln in lens:
        poffs.append(pos)
        pos += ln
    tile_len = pos
    host = np.empty(tile_len, dtype=np.uint8)
    for i, u in enumerate(order):
        host[poffs[i]:poffs[i] + lens[i]] = np.frombuffer(recs[u][0], dtype=np.uint8)
    tile = torch.from_numpy(host).to(dev)
    reps, rest = divmod(nblocks, period)
    rest_len = poffs[rest] if rest else 0
    parts = [tile.repeat(reps)] if reps else []
    if rest:
        parts.append(tile[:rest_len])
    parts.append(torch.zeros(64, dtype=torch.uint8, device=dev))
    d_frame = torch.cat(parts) if len(parts) > 1 else parts[0]
    del tile, parts, host
    frame_len = reps * tile_len + rest_len + 64
    descs = (lz4ada.BlockDesc * nblocks)()
    exp_hash = []
    comp_bytes = raw_bytes = 0
    for i in range(nblocks):
        q, j = divmod(i, period)
        u = order[j]
        rec, clen, rlen, h = recs[u][:4]
        d = descs[i]
        d.in_off = q * tile_len + poffs[j] + 4
        d.in_len = clen
        stored = (int.from_bytes(rec[:4], "little") >> 31) & 1
        has_ck = len(rec) == clen + 8
        d.flags = (lz4ada.BLOCK_STORED if stored else 0) | (lz4ada.BLOCK_HAS_CKSUM if has_ck else 0)
        d.out_off = i * (block_max + slot_pad)  # slot_pad: layout experiments only
        d.out_cap = block_max
        d.cksum = int.from_bytes(rec[4 + clen:8 + clen], "little") if has_ck else 0
        exp_hash.append(h)
        comp_bytes += clen
        raw_bytes += rlen
    d_desc = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(dev)
    if torch.device(dev).type == "cuda":
        torch.cuda.synchronize()
    return d_frame, frame_len, d_desc, exp_hash, comp_bytes, raw_bytes, descs


def med_ms(ev):
    """Median HIP-event time of a secondary row's repetitions (one stalled
    repetition on a shared box must not stand for the row; the headline's
    timed region keeps the contract's mean over exactly K steps)."""
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2]


def check_statuses(lz4ada, d_status, nblocks):
    return (lz4ada.BlockStatus * nblocks).from_buffer_copy(d_status.cpu().numpy().tobytes())


def golden_check(lz4ada, torch, d_status, descs, nb, op, dp, sp, d_hash, exp_hash, sh, what):
    st = check_statuses(lz4ada, d_status, nb)
    bad = [i for i in range(nb) if st[i].code != 0 or
           ((descs[i].flags & lz4ada.BLOCK_HAS_CKSUM) and st[i].cksum != descs[i].cksum)]
    assert not bad, f"{what}: block status / checksum errors: {bad[:5]}"
    lz4ada.output_checksums_device(op, dp, sp, nb, d_hash.data_ptr(), sh)
    torch.cuda.synchronize()
    got = [h & 0xffffffff for h in d_hash[:nb].cpu().tolist()]
    assert got == exp_hash, f"{what}: decoded output differs from the generator's plaintext"
    return st


# --------------------------------------------------------------- CPU baseline

def cpu_baseline_parallel(lz4frame, xxhash, recs, block_max, threads, blocks_per_thread):
    """SURVEY §8d's N-core extrapolation for independent frames: `threads`
    threads, each running the oracle's unlz4ada loop (ctypes releases the
    GIL) over its own frame of `blocks_per_thread` independent blocks of the
    same workload.  Reported beside cpu_baseline, never as it."""
    import concurrent.futures
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    frames = []
    for t in range(threads):
        blocks = [(recs[(t * blocks_per_thread + i) % len(recs)][4],
                   recs[(t * blocks_per_thread + i) % len(recs)][5], False)
                  for i in range(blocks_per_thread)]
        frames.append(lz4frame.build_frame(blocks, block_max, indep=True, block_cksum=True))

    L = O.lib()
    # output buffers and expected hashes outside the timed region; inside it
    # only the C loop runs (ctypes drops the GIL for the call)
    outs = [ctypes.create_string_buffer(len(raw) + MiB) for _, raw in frames]
    want = [xxhash.xxh32(raw).intdigest() for _, raw in frames]
    lens = [ctypes.c_int64() for _ in frames]

    def run(t):
        data, raw = frames[t]
        err = ctypes.create_string_buffer(512)
        st = L.oracle_unlz4ada(data, len(data), outs[t], len(raw) + MiB, ctypes.byref(lens[t]), err, 512)
        assert st == O.OK and lens[t].value == len(raw), err.value
        return len(raw)

    with concurrent.futures.ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        total = sum(ex.map(run, range(threads)))
        dt = time.perf_counter() - t0
    for t in range(threads):
        assert L.oracle_xxh32_hash(outs[t], lens[t].value) == want[t], "oracle output differs"
    return {"value": round(total / dt / MiB, 1), "unit": "MiB/s", "cores": threads, "kind": "port",
            "sample": f"{threads} threads x {blocks_per_thread} x 4 MiB blocks ({total / MiB:.0f} MiB "
                      f"decoded, {dt:.1f} s), one frame per thread through the oracle's unlz4ada "
                      "loop; block-parallel extrapolation for independent frames (SURVEY §8d)"}


def content_hash(xxhash, recs, nblocks, first=0):
    """Expected frame-wide XXH32 of a decoded shard (python-xxhash over the
    generator's plaintext, tiled like assemble_shard)."""
    h = xxhash.xxh32()
    for i in range(nblocks):
        h.update(recs[(first + i) % len(recs)][5])
    return h.intdigest()


def host_cpu_info(threads):
    """The host the CPU baselines ran on: CPU model, the machine's logical
    CPUs (nproc), the CPU share this job may use and the threads used."""
    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": affinity,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "threads_used": threads}


def cpu_baseline(lz4frame, xxhash, recs, block_max, budget_s):
    """The oracle (lz4ada.adb restated in C, 'port') through the reference's
    CLI loop (tool_unlz4ada: 4 KiB reads, one Update per call), one core,
    on a bounded prefix of the same frame."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O

    def frame_of(k):
        blocks = [(recs[i % len(recs)][4], recs[i % len(recs)][5], False) for i in range(k)]
        return lz4frame.build_frame(blocks, block_max, indep=True, block_cksum=True)
    L = O.lib()

    def timed(frame, raw):
        # the C loop alone: output buffer allocated, and the output checked,
        # outside the timed call
        out = ctypes.create_string_buffer(len(raw) + MiB)
        n = ctypes.c_int64()
        err = ctypes.create_string_buffer(512)
        t0 = time.perf_counter()
        st = L.oracle_unlz4ada(frame, len(frame), out, len(raw) + MiB, ctypes.byref(n), err, 512)
        dt = time.perf_counter() - t0
        assert st == O.OK and n.value == len(raw), err.value
        assert L.oracle_xxh32_hash(out, n.value) == xxhash.xxh32(raw).intdigest()
        return dt

    f1, raw1 = frame_of(1)
    t1 = timed(f1, raw1)
    k = max(1, min(2048, int(budget_s / max(t1, 1e-6))))
    fk, rawk = frame_of(k)
    dt = timed(fk, rawk)
    return {"value": round(len(rawk) / dt / MiB, 1), "unit": "MiB/s", "cores": 1,
            "kind": "port",
            "sample": f"{k} x 4 MiB blocks ({len(rawk) / MiB:.0f} MiB decoded, {dt:.1f} s) of the "
                      "same frame through the oracle's unlz4ada loop (4 KiB reads, Update per "
                      "call, block checksums verified)", "host": host_cpu_info(1)}


# ------------------------------------------------------------------ extra rows

def bench_class(M, dev, sh, stream, cls, nb, bmax, block_cksum=True, unique=16):
    """One more content class over the same layout, timed through the
    product call (block checksums when the frame has them + decode)."""
    lz4ada, lz4frame, xxhash, torch = M
    recs = make_unique_blocks(lz4ada, lz4frame, xxhash, cls, unique, bmax, block_cksum)
    fr, fl, de, eh, cb, rb, descs = assemble_shard(lz4ada, torch, recs, 0, nb, bmax, dev)
    d_out = torch.empty(nb * bmax, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(nb * 32, dtype=torch.uint8, device=dev)
    d_hash = torch.zeros(nb, dtype=torch.int32, device=dev)
    fp, dp, op, sp = fr.data_ptr(), de.data_ptr(), d_out.data_ptr(), d_st.data_ptr()
    lz4ada.decode_blocks_device(fp, fl, dp, nb, op, sp, sh)
    torch.cuda.synchronize()
    golden_check(lz4ada, torch, d_st, descs, nb, op, dp, sp, d_hash, eh, sh, cls)
    reps = 3
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        lz4ada.decode_blocks_device(fp, fl, dp, nb, op, sp, sh)
        b.record(stream)
    torch.cuda.synchronize()
    ms = med_ms(ev)
    # the decoder alone (no block checksums beside it)
    for a, b in ev:
        a.record(stream)
        lz4ada.launch_decode(fp, fl, dp, nb, op, sp, sh)
        b.record(stream)
    torch.cuda.synchronize()
    ms_dec = med_ms(ev)
    flg = 0x60 | (0x10 if block_cksum else 0)
    row = {"decode_ms": round(ms, 3), "MiB_s": round(rb / (ms * 1e-3) / MiB, 1),
           "frac": round((cb + rb) / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
           "decoder_alone_ms": round(ms_dec, 3),
           "decoder_alone_frac": round((cb + rb) / (ms_dec * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
           "ratio": round(cb / rb, 4), "flg": f"0x{flg:02x}", "blocks": nb,
           "compressed_bytes": cb, "decoded_bytes": rb,
           "golden": "per-block XXH32 of the output vs the generator"}
    del fr, de, d_out
    return row


# ------------------------------------------------- encoder-produced blocks
GOLDEN = os.path.join(ROOT, "tests", "golden")


def golden_recs(lz4ada, path, block_xxh32, raw_lens):
    """The blocks of a committed frame as make_unique_blocks records: (record
    bytes incl. size word [+ checksum], payload len, decoded len, decoded
    XXH32, payload, None).  The decoded digests come with the frame (the
    encoder's input, tests/golden/make_lz4_fixtures.py; or the frame's own
    content checksum), not from this repo's decoder or generator."""
    with open(path, "rb") as fh:
        data = fh.read()
    info, descs = lz4ada.frame_index(data)
    recs = []
    for i in range(info.nblocks):
        d = descs[i]
        has_ck = bool(d.flags & lz4ada.BLOCK_HAS_CKSUM)
        rec = data[d.in_off - 4:d.in_off + d.in_len + (4 if has_ck else 0)]
        recs.append((rec, d.in_len, raw_lens[i], block_xxh32[i], rec[4:4 + d.in_len], None))
    return recs


def real_sources(name):
    """(recs, description) of the real-data classes:
    t1111k -- the reference's densest test vector, one 4 MiB-BD block of
    1,137,664 decoded bytes (test_vectors_lz4/t1111k.lz4; golden: its frame's
    content checksum); liblz4_text -- the two 4 MiB blocks liblz4 1.9.3 made
    of 8 MiB of seeded text (tests/golden/lz4f/big4m.lz4; golden: the
    encoder input's per-block XXH32)."""
    import lz4ada
    if name == "t1111k":
        path = os.path.join(GOLDEN, "vectors", "t1111k.lz4")
        with open(path, "rb") as fh:
            data = fh.read()
        cc = int.from_bytes(data[-4:], "little")  # FLG 0x74: the content checksum ends the frame
        return golden_recs(lz4ada, path, [cc], [1137664]), \
            "reference vector t1111k (its one block, 222,593 sequences, ~5.1 B/sequence), tiled"
    ent = json.load(open(os.path.join(GOLDEN, "lz4f_digests.json")))["frames"]["big4m"]
    n = ent["input"]["len"]
    lens = [min(4 * MiB, n - i) for i in range(0, n, 4 * MiB)]
    return golden_recs(lz4ada, os.path.join(GOLDEN, "lz4f", "big4m.lz4"), ent["block_xxh32"], lens), \
        "liblz4 1.9.3 (level 1) blocks of seeded text (tests/golden/lz4f/big4m.lz4), tiled"


def match_sources(recs, hist=4080 + 16, cut_seq=128, cut_out=4080):
    """Where the decoder's matches read from, on these blocks: HBM (more than
    a batch + 16 bytes back, k_decode_idx's threshold), the LDS window (older
    than the batch), or this batch's own output -- under a model of the
    batch cut (128 sequences / 4,080 output bytes; the kernel cuts at 32-byte
    sub-segments).  Python parse of the unique blocks, outside any timing."""
    hbm = far = near = seqs = 0
    offs = []
    for rec in recs:
        b = rec[4]
        p, o, n = 0, 0, len(b)
        batch_o, batch_n = 0, 0
        while p < n:
            t = b[p]
            p += 1
            L = t >> 4
            if L == 15:
                while True:
                    e = b[p]
                    p += 1
                    L += e
                    if e != 255:
                        break
            p += L
            if p >= n:
                break
            off = b[p] | (b[p + 1] << 8)
            p += 2
            M = t & 15
            if M == 15:
                while True:
                    e = b[p]
                    p += 1
                    M += e
                    if e != 255:
                        break
            ml = M + 4
            if batch_n >= cut_seq or o + L + ml - batch_o > cut_out:
                batch_o, batch_n = o, 0
            batch_n += 1
            seqs += 1
            m = o + L
            if m - off < batch_o - hist:
                hbm += 1
            elif m - off + min(off, ml) <= batch_o:
                far += 1
            else:
                near += 1
            offs.append(off)
            o = m + ml
    tot = max(hbm + far + near, 1)
    offs.sort()
    return {"sequences": seqs, "matches": tot, "hbm_share": round(hbm / tot, 4),
            "window_share": round(far / tot, 4), "in_batch_share": round(near / tot, 4),
            "offset_median": offs[len(offs) // 2] if offs else 0,
            "offset_le_64_share": round(sum(1 for x in offs if x <= 64) / tot, 4),
            "model": "batch cut at 128 sequences / 4,080 output bytes; HBM = source more than "
                     "4,096 bytes before the batch"}


def bench_real(M, dev, sh, stream, name, bmax, target_bytes=8 << 30, reps=3):
    """A real-data class through the product call (block checksums beside
    the decode when the blocks carry them): the encoder's blocks tiled to
    ~8 GiB of output, golden per-block XXH32 against the frame's own
    digests."""
    lz4ada, lz4frame, xxhash, torch = M
    recs, what = real_sources(name)
    per = sum(r[2] for r in recs) / len(recs)
    nb = int(target_bytes // per)
    fr, fl, de, eh, cb, rb, descs = assemble_shard(lz4ada, torch, recs, 0, nb, bmax, dev)
    d_out = torch.empty(nb * bmax, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(nb * 32, dtype=torch.uint8, device=dev)
    d_hash = torch.zeros(nb, dtype=torch.int32, device=dev)
    fp, dp, op, sp = fr.data_ptr(), de.data_ptr(), d_out.data_ptr(), d_st.data_ptr()
    lz4ada.decode_blocks_device(fp, fl, dp, nb, op, sp, sh)
    torch.cuda.synchronize()
    golden_check(lz4ada, torch, d_st, descs, nb, op, dp, sp, d_hash, eh, sh, name)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        lz4ada.decode_blocks_device(fp, fl, dp, nb, op, sp, sh)
        b.record(stream)
    torch.cuda.synchronize()
    ms = med_ms(ev)
    for a, b in ev:
        a.record(stream)
        lz4ada.launch_decode(fp, fl, dp, nb, op, sp, sh)
        b.record(stream)
    torch.cuda.synchronize()
    ms_dec = med_ms(ev)
    row = {"data": what, "decode_ms": round(ms, 3), "MiB_s": round(rb / (ms * 1e-3) / MiB, 1),
           "frac": round((cb + rb) / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
           "decoder_alone_ms": round(ms_dec, 3),
           "decoder_alone_frac": round((cb + rb) / (ms_dec * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
           "ratio": round(cb / rb, 4), "blocks": nb, "kernel": lz4ada.bulk_decoder_kernel(nb),
           "compressed_bytes": cb, "decoded_bytes": rb,
           "match_sources": match_sources(recs),
           "golden": "per-block XXH32 of the output vs the frame's own digests (encoder input / "
                     "content checksum)"}
    # HBM traffic of k_decode_idx on this class (profiles/pmc_real.json, tools/pmc_real.sh:
    # FETCH_SIZE x 2 + WRITE_SIZE per launch of 2,048 blocks over the algorithmic bytes of that
    # launch), when the kernel's machine code is the one the counters were collected on
    try:
        pr = json.load(open(os.path.join(ROOT, "profiles", "pmc_real.json")))
        e = pr["classes"].get(name)
        if e and "traffic_over_alg" in e and pr.get("kernel_code_sha16") == kernel_code_hash("k_decode_idx"):
            row["traffic"] = {"hbm_bytes_per_launch": e["hbm_bytes_per_launch"],
                              "alg_bytes_per_launch": e["alg_bytes_per_launch"],
                              "traffic_over_alg": e["traffic_over_alg"],
                              "source": "profiles/pmc_real.json (2,048-block k_decode_idx launch)"}
    except (OSError, ValueError, KeyError):
        pass
    del fr, de, d_out
    return row


def bench_c3_one_gpu(M, dev, sh, stream, recs, bmax, nblocks=C3_BLOCKS, reps=3):
    """configs[3]'s whole frame (8192 x 4 MiB blocks, 32 GiB decoded) on ONE
    GPU -- the same-frame N=1 point of the 1->8 curve (N>1 lines split this
    frame over the ranks).  48 GiB of frame + output fit one MI355X's HBM."""
    lz4ada, lz4frame, xxhash, torch = M
    d_frame, frame_len, d_desc, exp_hash, comp, raw, descs = assemble_shard(
        lz4ada, torch, recs, 0, nblocks, bmax, dev)
    d_out = torch.empty(nblocks * bmax, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(nblocks * 32, dtype=torch.uint8, device=dev)
    d_hash = torch.zeros(nblocks, dtype=torch.int32, device=dev)
    fp, dp, op, sp = d_frame.data_ptr(), d_desc.data_ptr(), d_out.data_ptr(), d_st.data_ptr()
    lz4ada.decode_blocks_device(fp, frame_len, dp, nblocks, op, sp, sh)
    torch.cuda.synchronize()
    golden_check(lz4ada, torch, d_st, descs, nblocks, op, dp, sp, d_hash, exp_hash, sh, "c3 one GPU")
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(stream)
        lz4ada.decode_blocks_device(fp, frame_len, dp, nblocks, op, sp, sh)
        b.record(stream)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    ms = med_ms(ev)
    # one rank's share of the same frame at N = 2 / 4 / 8 (the first
    # 8192 / N blocks: every share holds whole periods of the 64 unique
    # blocks, so any rank's range has the same content), through the same
    # product call -- the per-rank compute time of the --gpus N lines, with
    # the library's own choice of decoder for that block count
    shares = {}
    for n in (2, 4, 8):
        nb = nblocks // n
        sev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(reps)]
        lz4ada.decode_blocks_device(fp, frame_len, dp, nb, op, sp, sh)
        for a, b in sev:
            a.record(stream)
            lz4ada.decode_blocks_device(fp, frame_len, dp, nb, op, sp, sh)
            b.record(stream)
        torch.cuda.synchronize()
        sms = med_ms(sev)
        shares[f"n{n}"] = {"blocks_per_rank": nb, "kernel_ms": round(sms, 3),
                           "decoder": lz4ada.bulk_decoder_kernel(nb),
                           "compute_only_efficiency": round(ms / (n * sms), 4)}
    st = check_statuses(lz4ada, d_st, nblocks // 8)
    assert all(x.code == 0 for x in st), "c3 share: block status"
    del d_frame, d_out, d_desc, d_st, d_hash
    torch.cuda.empty_cache()
    return {"workload": f"configs[3] frame on one GPU: {nblocks} x 4 MiB independent blocks = "
                        f"{raw >> 30} GiB decoded, FLG 0x70 (B.Indep|B.Checksum)",
            "blocks": nblocks, "kernel_ms": round(ms, 3), "wall_ms": round(wall * 1e3, 3),
            "value": round(raw / (wall) / MiB, 1), "unit": "MiB/s",
            "frac": round((comp + raw) / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
            "compressed_bytes": comp, "decoded_bytes": raw,
            "note": "same frame as the --gpus N>1 lines (strong scaling): N=1 point of the curve",
            "golden": "per-block XXH32 of the output vs the generator",
            "decoder": lz4ada.bulk_decoder_kernel(nblocks),
            "c3_shares": shares,
            "c3_shares_note": "one rank's shard of this frame at N=2/4/8 timed on this GPU (HIP "
                              "events, product call); compute_only_efficiency = kernel_ms(8192) / "
                              "(N x kernel_ms(share)): the strong-scaling ceiling before any "
                              "communication or host-side assembly"}


def bench_linked(M, dev, sh, stream, kind="mixed", nblocks=4096, bmax=256 * 1024, chain=64):
    """configs[4]: a linked frame (B.Indep = 0) of 4096 x 256 KiB blocks whose
    matches reach into the previous block: a chain of 64 generated blocks
    (each against the previous one's output), tiled -- the first block of
    the chain has no history references, so every tile boundary is valid."""
    import numpy as np
    lz4ada, lz4frame, xxhash, torch = M
    blocks = lz4ada.gen_linked_blocks(lz4ada.GEN_KINDS[kind], SEED0, bmax, chain)
    recs = [lz4frame.block_record(c, stored=False, block_cksum=True) for c, _ in blocks]
    hashes = [xxhash.xxh32(r).intdigest() for _, r in blocks]
    order = [i % chain for i in range(nblocks)]
    offs, pos = [], 0
    for u in order:
        offs.append(pos)
        pos += len(recs[u])
    host = np.zeros(pos + 64, dtype=np.uint8)
    arrs = [np.frombuffer(r, dtype=np.uint8) for r in recs]
    descs = (lz4ada.BlockDesc * nblocks)()
    comp = 0
    for i, u in enumerate(order):
        host[offs[i]:offs[i] + len(recs[u])] = arrs[u]
        clen = len(blocks[u][0])
        descs[i].in_off = offs[i] + 4
        descs[i].in_len = clen
        descs[i].flags = lz4ada.BLOCK_HAS_CKSUM
        descs[i].out_off = i * bmax
        descs[i].out_cap = bmax
        descs[i].cksum = int.from_bytes(recs[u][4 + clen:8 + clen], "little")
        comp += clen
    d_frame = torch.from_numpy(host).to(dev)
    raw = nblocks * bmax
    d_out = torch.empty(raw, dtype=torch.uint8, device=dev)

    def run():
        return lz4ada.decode_linked_device(d_frame.data_ptr(), pos + 64, descs, nblocks, bmax,
                                           d_out.data_ptr(), raw, sh)
    run()  # warmup (allocator, code objects)
    reps = 3
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        n = run()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    assert n == raw, "linked frame: decoded length differs"
    # golden: per-block XXH32 of the contiguous output (every block is full)
    st = (lz4ada.BlockStatus * nblocks)()
    for i in range(nblocks):
        st[i].out_len = bmax
    d_desc = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(dev)
    d_st = torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8).to(dev)
    d_hash = torch.zeros(nblocks, dtype=torch.int32, device=dev)
    lz4ada.output_checksums_device(d_out.data_ptr(), d_desc.data_ptr(), d_st.data_ptr(), nblocks,
                                   d_hash.data_ptr(), sh)
    torch.cuda.synchronize()
    got = [h & 0xffffffff for h in d_hash.cpu().tolist()]
    assert got == [hashes[u] for u in order], "linked frame: decoded output differs"
    del d_frame, d_out
    return {"workload": f"configs[4]: linked frame (FLG 0x50: B.Checksum, B.Indep=0), {nblocks} x "
                        f"{bmax >> 10} KiB {kind} blocks, matches reach into the previous block",
            "decode_ms": round(ms, 3), "MiB_s": round(raw / (ms * 1e-3) / MiB, 1),
            "frac": round((comp + raw) / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
            "compressed_bytes": comp, "decoded_bytes": raw,
            "path": "lz4ada_decode_linked_device: block checksums (side stream), k_index, "
                    "k_decode_idx_lk + k_decode_idx_zl concurrently (every block at once: history "
                    "plane X = k & 255, plane Z with literals 0 and history k >> 8; quirk D1 emulated "
                    "under the predicted round state; a third plane only for blocks flagged deep), k_link_init (words and bytes) + k_link_jump rounds (history "
                    "resolved on the GPU); wall clock of the whole call, device-resident frame "
                    "and output",
            "golden": "per-block XXH32 of the output vs the generator"}


def bench_64k(M, dev, sh, stream, kind="mixed", nblocks=16384, bmax=64 * 1024, unique=64):
    """configs[1]: a 1 GiB frame of 64 KiB independent blocks with a content
    checksum.  The decode launch (block checksums + decode, device-resident)
    is timed with HIP events; the frame-wide content XXH32 (one serial chain,
    SURVEY H2) runs through the D2H + host-chain pipeline and is reported
    beside it."""
    lz4ada, lz4frame, xxhash, torch = M
    recs = make_unique_blocks(lz4ada, lz4frame, xxhash, kind, unique, bmax)
    d_frame, frame_len, d_desc, exp_hash, comp, raw, descs = assemble_shard(
        lz4ada, torch, recs, 0, nblocks, bmax, dev)
    d_out = torch.empty(nblocks * bmax, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(nblocks * 32, dtype=torch.uint8, device=dev)
    d_hash = torch.zeros(nblocks, dtype=torch.int32, device=dev)
    fp, dp, op, sp = d_frame.data_ptr(), d_desc.data_ptr(), d_out.data_ptr(), d_st.data_ptr()
    lz4ada.decode_blocks_device(fp, frame_len, dp, nblocks, op, sp, sh)
    torch.cuda.synchronize()
    golden_check(lz4ada, torch, d_st, descs, nblocks, op, dp, sp, d_hash, exp_hash, sh, "64 KiB")
    reps = 5
    e0, e1, e2, e3 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
    e0.record(stream)
    for _ in range(reps):
        lz4ada.decode_blocks_device(fp, frame_len, dp, nblocks, op, sp, sh)
    e1.record(stream)
    for _ in range(reps):
        lz4ada.launch_block_checksums(fp, dp, nblocks, sp, sh)
    e2.record(stream)
    for _ in range(reps):
        lz4ada.launch_decode(fp, frame_len, dp, nblocks, op, sp, sh)
    e3.record(stream)
    torch.cuda.synchronize()
    step_ms = e0.elapsed_time(e1) / reps
    ck_ms, dec_ms = e1.elapsed_time(e2) / reps, e2.elapsed_time(e3) / reps
    h = lz4ada.XXHash32()
    t0 = time.perf_counter()
    h.update_device_d2h(op, raw, None, sh)
    t_hash = time.perf_counter() - t0
    assert h.final() == content_hash(xxhash, recs, nblocks), "64 KiB frame content checksum"
    del d_frame, d_out
    return {"workload": f"configs[1]: {raw >> 30} GiB frame, {nblocks} x 64 KiB independent "
                        f"{kind} blocks, FLG 0x74 (B.Indep|B.Checksum|C.Checksum)",
            "step_ms": round(step_ms, 3), "decode_alone_ms": round(dec_ms, 3),
            "checksum_alone_ms": round(ck_ms, 3),
            "MiB_s": round(raw / (step_ms * 1e-3) / MiB, 1),
            "frac": round((comp + raw) / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
            "content_xxh32_s": round(t_hash, 3),
            "e2e_MiB_s": round(raw / (step_ms * 1e-3 + t_hash) / MiB, 1),
            "compressed_bytes": comp, "decoded_bytes": raw}


def bench_facade(feed=4096, reps=5):
    """the streaming facade (Init_With_Header + Update)
    driven from C the way tool_unlz4ada drives the library -- 4 KiB reads
    (tool_unlz4ada/unlz4ada.adb:16, 84-103), a context per frame -- on three
    frames with block and content checksums: 64 KiB independent blocks (the
    LZ4F default block size), 64 KiB linked blocks (the LZ4F default frame:
    linked, 64 KiB), 256 KiB linked blocks, 4 MiB independent blocks.  Each is timed next to the oracle's 1-core loop over the same
    frame (the reference's CPU path, 4 KiB reads).  Host-resident input and
    output: this is the facade's latency path, not the bulk roofline."""
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    import lz4ada
    import lz4frame
    exe = os.path.join(ROOT, "bo-lz4-ada_amd", "facade_bench")
    L = O.lib()
    # linked_64k_d1: uniform offsets up to 65,535, so matches >= 65,529 back
    # meet quirk D1 (lib/lz4ada.adb:811-817, 862-879) in many blocks
    cases = [("indep_64k", 64 << 10, 64, True, "mixed"), ("linked_64k", 64 << 10, 64, False, "mixed_nod1"),
             ("linked_64k_d1", 64 << 10, 64, False, "mixed"),
             ("linked_256k", 256 << 10, 32, False, "mixed_nod1"), ("indep_4m", 4 << 20, 8, True, "mixed")]
    rows = {}
    with tempfile.TemporaryDirectory() as td:
        for name, bmax, nb, indep, kind in cases:
            if indep:
                blocks = [(*lz4ada.gen_block(lz4ada.GEN_KINDS[kind], SEED0 + i, bmax), False)
                          for i in range(nb)]
            else:  # mixed_nod1: offsets below 65529, no block meets quirk D1
                blocks = [(c, r, False) for c, r in
                          lz4ada.gen_linked_blocks(lz4ada.GEN_KINDS[kind], SEED0, bmax, nb)]
            # (the reference's D1 bytes differ from the encoder input, so a
            # content checksum over the input would fail: none on that frame)
            frame, _ = lz4frame.build_frame(blocks, bmax, indep=indep, block_cksum=True,
                                            content_cksum=name != "linked_64k_d1")
            st, expect, msg = O.unlz4ada(frame, out_cap=len(frame) * 4 + (8 << 20))
            assert st == O.OK, msg
            path = os.path.join(td, name + ".lz4")
            with open(path, "wb") as fh:
                fh.write(frame)
            with open(path + ".out", "wb") as fh:
                fh.write(expect)
            r = subprocess.run([exe, path, str(feed), str(reps)], capture_output=True, text=True,
                               timeout=300)
            assert r.returncode == 0, f"facade_bench {name}: {r.stderr[-500:]}"
            row = json.loads(r.stdout.strip().splitlines()[-1])
            # the oracle's loop over the same frame, best of three
            out = ctypes.create_string_buffer(len(expect) + (1 << 20))
            n = ctypes.c_int64()
            err = ctypes.create_string_buffer(512)
            best = None
            for _ in range(3):
                t0 = time.perf_counter()
                st = L.oracle_unlz4ada(frame, len(frame), out, len(expect) + (1 << 20),
                                       ctypes.byref(n), err, 512)
                dt = time.perf_counter() - t0
                assert st == O.OK and n.value == len(expect)
                best = dt if best is None else min(best, dt)
            row["oracle_1core_mib_s"] = round(len(expect) / best / MiB, 1)
            cks = "block checksum" if name == "linked_64k_d1" else "block + content checksum"
            row["frame"] = (f"{nb} x {bmax >> 10} KiB {'independent' if indep else 'linked'} {kind} "
                            f"blocks, {cks}, {len(expect) / MiB:.0f} MiB decoded")
            rows[name] = row
    rows["bulk_linked_64k_d1"] = bench_d1_frame()
    rows["note"] = (f"bo-lz4-ada_amd/facade_bench: {feed}-byte Update calls from C, median of {reps} "
                    "frames, a context per frame, output checked; oracle_1core_mib_s: the oracle's "
                    "unlz4ada loop over the same frame (1 core)")
    return rows


def bench_d1_frame(nb=256, reps=5):
    """256 linked 64 KiB blocks with uniform offsets
    (quirk D1 in many blocks) through lz4ada_decode_frame from host memory,
    output equal to the oracle's (the reference's bytes, D1 included);
    median of `reps`, and which paths ran (lz4ada_last_path)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    import lz4ada
    import lz4frame
    blocks = lz4ada.gen_linked_blocks(lz4ada.GEN_KINDS["mixed"], 0x4C5A3441, 64 << 10, nb)
    frame, _ = lz4frame.build_frame([(c, r, False) for c, r in blocks], 64 << 10, indep=False)
    st, ref, msg = O.unlz4ada(frame, out_cap=nb * (64 << 10) + (1 << 20))
    assert st == O.OK, msg
    lz4ada.decode_frame(frame)  # warm
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out, used = lz4ada.decode_frame(frame)
        ts.append(time.perf_counter() - t0)
        assert out == ref and used == len(frame)
    ts.sort()
    t = ts[len(ts) // 2]
    return {"ms": round(t * 1e3, 2), "mib_s": round(len(ref) / t / MiB, 1), "path": lz4ada.last_path(),
            "frame": f"{nb} x 64 KiB linked mixed blocks (uniform offsets), no checksums, host in/out",
            "note": "lz4ada_decode_frame, median of %d; path bits: 2 linked bulk, 4 exact resume" % reps}


# ----------------------------------------------------------------------- main

def launch_check(args):
    """--launch-check: the rank side of the launcher test (gloo, no GPU)."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
        lo, hi = shard_range(rank, world, args.blocks or C3_BLOCKS)
        import torch
        t = torch.tensor([hi - lo], dtype=torch.int64)
        dist.all_reduce(t)
        total = int(t.item())
        dist.destroy_process_group()
    else:
        total = args.blocks or 2048
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks": world, "blocks_total": total}), flush=True)


def shard_range(rank, world, total):
    """Contiguous block range [lo, hi) of `rank` (configs[3]'s split)."""
    lo = total * rank // world
    hi = total * (rank + 1) // world
    return lo, hi


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if args.launch_check:
        return launch_check(args)

    import torch  # noqa: E402  (torch's HIP runtime before liblz4ada_hip.so)
    import torch.distributed as dist  # noqa: E402
    import xxhash  # noqa: E402
    import lz4ada  # noqa: E402
    import lz4frame  # noqa: E402
    M = (lz4ada, lz4frame, xxhash, torch)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        assert dist.get_world_size() == world
        if args.gpus not in (1, world):
            raise SystemExit(f"--gpus {args.gpus} but the launcher started {world} ranks")
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    bmax = args.block_max
    total_blocks = args.blocks or (2048 if world == 1 else C3_BLOCKS)
    lo, hi = shard_range(rank, world, total_blocks)
    nb = hi - lo
    log(f"[bench] {world} rank(s), frame of {total_blocks} x {bmax >> 20} MiB blocks; "
        f"generating {args.unique} unique {args.kind} blocks ...")
    recs = make_unique_blocks(lz4ada, lz4frame, xxhash, args.kind, args.unique, bmax)
    d_frame, frame_len, d_desc, exp_hash, comp_bytes, raw_bytes, descs = assemble_shard(
        lz4ada, torch, recs, lo, nb, bmax, dev)
    d_out = torch.empty(nb * bmax, dtype=torch.uint8, device=dev)
    d_status = torch.zeros(nb * 32, dtype=torch.uint8, device=dev)
    d_hash = torch.zeros(nb, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    fp, dp, op, sp = d_frame.data_ptr(), d_desc.data_ptr(), d_out.data_ptr(), d_status.data_ptr()
    log(f"[bench] rank shard: blocks [{lo}, {hi}), {comp_bytes / MiB:.0f} MiB compressed -> "
        f"{raw_bytes / MiB:.0f} MiB decoded")

    def step(events=None):
        # the product call: block checksums on the library's side stream
        # beside the decoder's first pass, joined back into `stream`
        if events is not None:
            events[0].record(stream)
        lz4ada.decode_blocks_device(fp, frame_len, dp, nb, op, sp, sh)
        if events is not None:
            events[1].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # ---- golden check (outside the timed region)
    st = golden_check(lz4ada, torch, d_status, descs, nb, op, dp, sp, d_hash, exp_hash, sh,
                      "headline")
    assert sum(s.out_len for s in st) == raw_bytes
    log("[bench] golden check passed (per-block XXH32 of output, block checksums)")

    # ---- timed region: exactly K steps
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed)
    dec_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    # the one status collective (all-reduce MAX of the block
    # statuses), after the timed region
    st = check_statuses(lz4ada, d_status, nb)
    local_bad = int(any(s.code != 0 for s in st))
    if world > 1:
        t = torch.tensor([local_bad], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        local_bad = int(t.item())
    assert local_bad == 0
    # the two halves alone (after the timed region, same stream): what the
    # overlap hides
    alone = {}
    for name, fn in (("block_checksums", lambda: lz4ada.launch_block_checksums(fp, dp, nb, sp, sh)),
                     ("decode", lambda: lz4ada.launch_decode(fp, frame_len, dp, nb, op, sp, sh))):
        a_ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(3)]
        for a, b in a_ev:
            a.record(stream)
            fn()
            b.record(stream)
        torch.cuda.synchronize()
        alone[name] = round(sum(a.elapsed_time(b) for a, b in a_ev) / len(a_ev), 3)

    ms_per_step = elapsed / args.steps * 1e3
    # the whole frame's bytes (every rank's shard; the tiling is deterministic)
    total_raw = sum(recs[i % len(recs)][2] for i in range(total_blocks))
    frame_alg = total_raw + sum(recs[i % len(recs)][1] for i in range(total_blocks))
    value = total_raw * args.steps / elapsed / MiB
    dec_kernel = lz4ada.bulk_decoder_kernel(nb)  # the kernel this block count runs
    alg_bytes = comp_bytes + raw_bytes  # compressed read once + output written once
    achieved = alg_bytes / (dec_ms * 1e-3) / 1e9
    traffic = None
    traffic_src = None
    if os.path.exists(args.pmc):
        with open(args.pmc) as fh:
            pmc = json.load(fh)
        # only a figure measured on this workload with this kernel's code
        code = kernel_code_hash(dec_kernel)
        if (pmc.get("config") == {"kind": args.kind, "blocks": nb, "block_max": bmax}
                and pmc.get("kernel") == dec_kernel and code is not None
                and pmc.get("kernel_code_sha16") == code):
            traffic = pmc.get("hbm_bytes_per_launch")
            traffic_src = pmc.get("source")
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
            "kernel": dec_kernel, "kernel_ms": round(dec_ms, 3),
            "kernel_ms_note": "HIP events (rank 0) around lz4ada_decode_blocks_device on its "
                              "stream: k_decode_idx (pass 1 then pass 2 of each block in one "
                              "wave) with k_xxh32_rows (block checksums) overlapped on the side "
                              "stream",
            "alg_bytes_per_launch": alg_bytes,
            "traffic_source": traffic_src, "kernel_code_sha16": kernel_code_hash(dec_kernel),
            "alone_ms": alone}

    if world > 1:
        workload = (f"configs[3]: {total_blocks * bmax >> 30} GiB frame, {total_blocks} x 4 MiB "
                    f"independent blocks, FLG 0x70 (B.Indep|B.Checksum), BD 0x70, split into "
                    f"{world} contiguous block ranges (one per GPU)")
    else:
        workload = (f"configs[2] size, configs[3] shape: {total_blocks} x 4 MiB independent "
                    f"blocks = {raw_bytes >> 30} GiB decoded, FLG 0x70 (B.Indep|B.Checksum), "
                    "BD 0x70 (content-checksum variant FLG 0x74: e2e_content_checksum)")
    result = {
        "metric": METRIC, "value": round(value, 1), "unit": "MiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True, "scaling": "strong",
        "scaling_note": "N>1: configs[3]'s 32 GiB frame split over the ranks (total work fixed; "
                        "its same-frame N=1 point is c3_one_gpu); N=1: the 8 GiB configs[2]-size frame",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: repo LZ4 sequence generator, 64 unique blocks tiled in host memory",
        "config": {"workload": workload, "class": args.kind, "blocks_total": total_blocks,
                   "blocks_per_gpu": nb, "block_max": bmax,
                   "compressed_bytes_rank0": comp_bytes, "decoded_bytes_rank0": raw_bytes,
                   "parallelism": f"block-shard x{world}"},
        "hbm_gbps_step": round(frame_alg / (elapsed / args.steps) / 1e9, 1),
        "roofline": roof,
    }
    if world > 1:
        result["rccl_ranks"] = dist.get_world_size()
        # every rank's block count and decode time (HIP events on its stream)
        mine = torch.tensor([float(nb), dec_ms, elapsed / args.steps * 1e3], dtype=torch.float64,
                            device=dev)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        result["per_rank"] = [{"rank": r, "blocks_per_gpu": int(t[0].item()),
                               "kernel_ms": round(float(t[1].item()), 3)}
                              for r, t in enumerate(allr)]

    extra = world == 1 and rank == 0
    # ---- configs[2] e2e: + frame-wide content XXH32 (one serial chain), run
    # by the D2H + host-chain pipeline (lz4ada_content_xxh32_d2h) the bulk
    # path uses: chunks are hashed while the next one is in flight
    if extra and not args.no_e2e:
        h = lz4ada.XXHash32()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h.update_device_d2h(op, raw_bytes, None, sh)
        t_hash = time.perf_counter() - t0
        assert h.final() == content_hash(xxhash, recs, nb), "content checksum mismatch"
        result["e2e_content_checksum"] = {
            "workload": "configs[2]: same 8 GiB frame with FLG 0x74 (+C.Checksum)",
            "content_xxh32_s": round(t_hash, 3),
            "value": round(raw_bytes / (ms_per_step * 1e-3 + t_hash) / MiB, 1), "unit": "MiB/s",
            "note": "frame-wide XXH32 is one serial 4-lane chain (SURVEY H2): decoded bytes "
                    "stream to the host in 32 MiB chunks, each hashed by one host core while "
                    "the next is in flight (one GPU wave runs the chain at ~1.1 GB/s)"}

    # ---- configs[3]'s frame on this one GPU (the curve's same-frame N=1 point)
    if extra and not args.no_c3:
        del d_out, d_frame
        torch.cuda.empty_cache()
        log("[bench] c3_one_gpu (8192 x 4 MiB on one GPU) ...")
        result["c3_one_gpu"] = bench_c3_one_gpu(M, dev, sh, stream, recs, bmax)
        d_out = None

    # ---- other content classes through the product call, same layout
    if extra:
        del d_out
        rows = {}
        for cls in [c for c in args.classes.split(",") if c]:
            log(f"[bench] class {cls} ...")
            if cls == "stored":
                # README.md:753-766's `random` rows: lz4 CLI defaults, no block checksum
                rows["stored"] = bench_class(M, dev, sh, stream, "stored", nb, bmax, block_cksum=False)
                rows["stored_bcksum"] = bench_class(M, dev, sh, stream, "stored", nb, bmax)
            else:
                rows[cls] = bench_class(M, dev, sh, stream, cls, nb, bmax)
        for name in [c for c in args.real.split(",") if c]:
            log(f"[bench] real-data class {name} ...")
            torch.cuda.empty_cache()
            rows[name] = bench_real(M, dev, sh, stream, name, bmax)
        if rows:
            result["classes"] = rows

    # ---- configs[4]: linked (dependent) 256 KiB-block frame, 1 GiB, one GPU:
    # every block at once against synthetic history, resolved on the GPU
    if extra and not args.no_linked:
        log("[bench] configs[4] linked row ...")
        result["linked_c5"] = bench_linked(M, dev, sh, stream)
    # ---- configs[1]: 1 GiB of 64 KiB independent blocks + content checksum
    if extra and not args.no_64k:
        log("[bench] configs[1] 64 KiB row ...")
        result["c2_64k"] = bench_64k(M, dev, sh, stream)

    # ---- the streaming facade at tool_unlz4ada's 4 KiB reads
    if extra and not args.no_facade:
        log("[bench] facade (4 KiB reads from C) ...")
        torch.cuda.empty_cache()
        result["facade"] = bench_facade()

    if extra and not args.no_cpu_baseline:
        log("[bench] CPU baseline (oracle) ...")
        result["cpu_baseline"] = cpu_baseline(lz4frame, xxhash, recs, bmax, args.cpu_budget)
        # the GPU box's CPU share is 16 cores (OMP_NUM_THREADS there; nproc and
        # os.cpu_count() show the whole machine's): one oracle thread per core
        share = int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)
        threads = min(share, os.cpu_count() or 1)
        par = cpu_baseline_parallel(lz4frame, xxhash, recs, bmax, threads, 64)
        par["host"] = host_cpu_info(threads)
        result["cpu_baseline_parallel"] = par
    elif rank == 0:
        result["cpu_baseline"] = None

    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
