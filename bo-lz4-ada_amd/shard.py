"""Multi-GPU sharding of independent-block frames.

One process per GPU (torch.distributed, RCCL over xGMI for the few small
collectives).  A frame whose blocks are independent (FLG.B.Indep) is split
into contiguous block ranges, balanced by compressed bytes; each rank copies
only its range of the compressed frame to its GPU and decodes it with
``lz4ada_decode_blocks_device`` -- no data-path collective.  Then:

* the ranks agree on one block status with a single ``all_reduce(MAX)``;
* the frame-level checks of ``Check_End_Mark`` (lz4ada.adb:463-523) run
  across ranks: the declared content size against the ``all_reduce(SUM)``
  of the decoded lengths, and the content checksum as ONE XXH32 chain in
  frame order -- rank r receives the running 48-byte hasher state from
  rank r-1, hashes its own decoded bytes (D2H + host chain,
  ``lz4ada_content_xxh32_d2h``), and passes it on; the last rank's Final
  value is broadcast.  The chain is serial by nature.

On any failure every rank re-runs the frame through the single-GPU path
(``lz4ada.decode_frame``) so it raises the reference's exception and message
-- the same decision on every rank.

Linked frames (B.Indep = 0) do not shard: they decode on one GPU
("replicas only").
"""
import ctypes
from typing import Callable, List, Sequence, Tuple

import lz4ada  # noqa: F401  (imports torch first: one HIP runtime)
import torch
import torch.distributed as dist

# status codes carried by the all-reduce (0 = every block fine)
SHARD_OK = 0
SHARD_BLOCK_ERROR = 1


def plan_shards(in_lens: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous block ranges [lo, hi) per rank, balanced by compressed bytes.

    Rank r takes the blocks whose compressed prefix midpoint falls in
    [r, r+1) * total / world; every block goes to exactly one rank and the
    ranges are in frame order (a rank may get an empty range when there are
    fewer blocks than ranks)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    n = len(in_lens)
    total = sum(int(x) for x in in_lens)
    bounds = [0] * (world + 1)
    bounds[world] = n
    acc = 0
    r = 1
    for i, ln in enumerate(in_lens):
        mid2 = 2 * acc + int(ln)  # 2 * midpoint, avoids fractions
        while r < world and mid2 * world >= 2 * r * total:
            bounds[r] = i
            r += 1
        acc += int(ln)
    while r < world:
        bounds[r] = n
        r += 1
    return [(bounds[k], bounds[k + 1]) for k in range(world)]


def shard_slice(descs, lo: int, hi: int):
    """Byte range of the compressed frame a rank needs for blocks [lo, hi),
    and the descriptors re-based to that slice and to a dense output buffer.

    Returns (byte_lo, byte_hi, local_descs (ctypes array), out_bytes)."""
    k = hi - lo
    local = (lz4ada.BlockDesc * max(k, 1))()
    if k == 0:
        return 0, 0, local, 0
    b0 = descs[lo].in_off
    b1 = max(descs[i].in_off + descs[i].in_len for i in range(lo, hi))
    out_base = descs[lo].out_off
    out_end = 0
    for j, i in enumerate(range(lo, hi)):
        d = descs[i]
        local[j].in_off = d.in_off - b0
        local[j].in_len = d.in_len
        local[j].flags = d.flags
        local[j].out_off = d.out_off - out_base
        local[j].out_cap = d.out_cap
        local[j].cksum = d.cksum
        out_end = max(out_end, local[j].out_off + d.out_cap)
    return b0, b1, local, out_end


def block_errors(descs, statuses) -> List[int]:
    """Indices of blocks the bulk path rejects: a device status or a block
    checksum mismatch (lz4ada.adb:672-676)."""
    bad = []
    for i, (d, s) in enumerate(zip(descs, statuses)):
        if s.code != 0 or ((d.flags & lz4ada.BLOCK_HAS_CKSUM) and s.cksum != d.cksum):
            bad.append(i)
    return bad


def _dist_on() -> bool:
    return dist.is_available() and dist.is_initialized()


def reduce_status(local: int, group=None, device=None) -> int:
    """The one status collective: MAX of the per-rank status."""
    if not _dist_on():
        return local
    t = torch.tensor([local], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def reduce_sum(local: int, group=None, device=None) -> int:
    """SUM over ranks (decoded bytes, for the declared content size)."""
    if not _dist_on():
        return local
    t = torch.tensor([local], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return int(t.item())


def _global(group, r: int) -> int:
    return dist.get_global_rank(group, r) if group is not None else r


XXH32_EMPTY = 0x02CC5D05  # XXH32 of no bytes, seed 0 (vector `empty`)


def chain_xxh32(init: bytes, update_local: Callable[[bytes], bytes],
                finalize: Callable[[bytes], int], rank: int, world: int, group=None,
                device=None) -> int:
    """ONE XXH32 chain over every rank's bytes in rank order (a frame-wide
    content checksum, lz4ada.adb:709-714, 493-501).  The hasher state is an
    opaque byte string: rank 0 starts from `init`, every rank applies
    `update_local` to the state it receives from rank-1 and sends the result
    to rank+1; the last rank's `finalize` value is broadcast to all."""
    if world > 1 and not _dist_on():
        raise ValueError("a content checksum across ranks needs an initialised process group")
    state = init
    if rank > 0:
        t = torch.empty(len(init), dtype=torch.uint8, device=device)
        dist.recv(t, src=_global(group, rank - 1), group=group)
        state = bytes(t.cpu().numpy().tobytes())
    state = update_local(state)
    if rank + 1 < world:
        t = torch.frombuffer(bytearray(state), dtype=torch.uint8).to(device)
        dist.send(t, dst=_global(group, rank + 1), group=group)
    h = finalize(state) if rank == world - 1 else 0
    if world > 1:
        t = torch.tensor([h], dtype=torch.int64, device=device)
        dist.broadcast(t, src=_global(group, world - 1), group=group)
        h = int(t.item())
    return h


def _device_runs(local, k: int, out_lens: Sequence[int]):
    """(offset, length) runs of consecutive decoded bytes in a rank's slots."""
    runs = []
    for j in range(k):
        off, n = local[j].out_off, int(out_lens[j])
        if runs and runs[-1][0] + runs[-1][1] == off:
            runs[-1] = (runs[-1][0], runs[-1][1] + n)
        elif n:
            runs.append((off, n))
    return runs


def _product_hasher(d_out, runs, stream: int):
    """update_local / finalize over the product's hasher state: the rank's
    decoded bytes stream to the host chain (lz4ada_content_xxh32_d2h)."""
    size = ctypes.sizeof(lz4ada.XXH32State)

    def update(state: bytes) -> bytes:
        st = lz4ada.XXH32State.from_buffer_copy(state)
        for off, n in runs:
            lz4ada._check(lz4ada._lib.lz4ada_content_xxh32_d2h(
                ctypes.byref(st), d_out.data_ptr() + off, n, None, stream), lz4ada._thread_error())
        return bytes(st)[:size]

    def final(state: bytes) -> int:
        st = lz4ada.XXH32State.from_buffer_copy(state)
        return st.hash if st.total_length else XXH32_EMPTY

    init = lz4ada.XXH32State()
    lz4ada._lib.lz4ada_xxh32_reset(ctypes.byref(init), 0)
    return bytes(init)[:size], update, final


def frame_checks_ok(info, total_local: int, hasher, rank: int, world: int, group=None,
                    device=None) -> bool:
    """Check_End_Mark's frame-level checks across ranks (lz4ada.adb:463-523):
    declared content size vs the summed decoded bytes, and the content
    checksum chained in frame order.  Same answer on every rank."""
    if world > 1 and not _dist_on() and (info.has_content_size or info.content_checksum):
        raise ValueError("frame-level checks across ranks need an initialised process group")
    total = reduce_sum(total_local, group, device)
    if info.has_content_size and total != info.content_size:
        return False
    if info.content_checksum:
        init, update, final = hasher()
        if chain_xxh32(init, update, final, rank, world, group, device) != \
                info.content_checksum_declared:
            return False
    return True


def decode_frame_sharded(frame: bytes, rank: int, world: int, device, group=None,
                         coll_device=None):
    """Decode this rank's share of an independent-block frame on `device`.

    Returns (d_out uint8 tensor, (lo, hi) block range, out_lens list).  The
    output stays resident on the rank's GPU (slots of block_max bytes).
    Raises the reference exception (via the exact path) if any rank found a
    bad block or the frame-level checks fail; linked frames raise ValueError
    (they do not shard).  A frame with B.Indep set whose blocks read earlier
    blocks decodes, as the reference decodes it, through the
    one-GPU linked path: rank 0 returns it whole as one run ((0, nblocks),
    [length]), the other ranks an empty range.  coll_device: device of the collectives' tensors
    (default `device`; "cpu" for a gloo group)."""
    coll = coll_device if coll_device is not None else device
    info, descs = lz4ada.frame_index(frame)
    if info.format != lz4ada.FORMAT_MODERN or not info.independent:
        raise ValueError("only independent-block modern frames shard")
    ranges = plan_shards([descs[i].in_len for i in range(info.nblocks)], world)
    lo, hi = ranges[rank]
    b0, b1, local, out_bytes = shard_slice(descs, lo, hi)
    k = hi - lo
    d_out = torch.empty(max(out_bytes, 1), dtype=torch.uint8, device=device)
    status = SHARD_OK
    out_lens: List[int] = []
    stream = torch.cuda.current_stream(device)
    if k:
        d_in = torch.frombuffer(bytearray(frame[b0:b1]), dtype=torch.uint8).to(device)
        d_desc = torch.frombuffer(bytearray(bytes(local)[:k * ctypes.sizeof(lz4ada.BlockDesc)]),
                                  dtype=torch.uint8).to(device)
        d_st = torch.zeros(k * ctypes.sizeof(lz4ada.BlockStatus), dtype=torch.uint8,
                           device=device)
        lz4ada.decode_blocks_device(d_in.data_ptr(), b1 - b0, d_desc.data_ptr(), k,
                                    d_out.data_ptr(), d_st.data_ptr(), stream.cuda_stream)
        stream.synchronize()
        raw = d_st.cpu().numpy().tobytes()
        sts = (lz4ada.BlockStatus * k).from_buffer_copy(raw)
        if block_errors([local[j] for j in range(k)], sts):
            status = SHARD_BLOCK_ERROR
        out_lens = [s.out_len for s in sts]
    ok = reduce_status(status, group, coll) == SHARD_OK
    if ok:
        runs = _device_runs(local, k, out_lens)
        ok = frame_checks_ok(info, sum(out_lens),
                             lambda: _product_hasher(d_out, runs, stream.cuda_stream),
                             rank, world, group, coll)
    if not ok:
        out, _ = lz4ada.decode_frame(frame)  # raises the reference exception
        # the single-GPU path accepted it: a block reaches before its own
        # start (B.Indep set but ignored by the reference) ->
        # linked data, decoded by the linked path.  It does not shard: rank 0
        # holds the whole output as one run, the other ranks nothing.
        n = info.nblocks
        if rank != 0:
            return torch.empty(1, dtype=torch.uint8, device=device), (n, n), []
        d = torch.frombuffer(bytearray(out or b"\0"), dtype=torch.uint8).to(device)
        return d, (0, n), [len(out)]
    return d_out, (lo, hi), out_lens
