"""Multi-GPU sharding of independent-block frames.

One process per GPU (torch.distributed, RCCL over xGMI for the one
collective).  A frame whose blocks are independent (FLG.B.Indep) is split
into contiguous block ranges, balanced by compressed bytes; each rank copies
only its range of the compressed frame to its GPU and decodes it with
``lz4ada_decode_blocks_device`` — no data-path collective.  The ranks agree
on one error status with a single ``all_reduce(MAX)``; on any error every
rank re-runs the frame through the exact single-GPU path
(``lz4ada.decode_frame``) so it raises the reference's exception and message
(lz4ada.adb:661-707 error precedence) — the same decision on every rank.

Linked frames (B.Indep = 0) do not shard: they decode on one GPU
("replicas only").
"""
import ctypes
from typing import List, Sequence, Tuple

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


def reduce_status(local: int, group=None, device=None) -> int:
    """The one collective: MAX of the per-rank status."""
    if not dist.is_available() or not dist.is_initialized():
        return local
    t = torch.tensor([local], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def decode_frame_sharded(frame: bytes, rank: int, world: int, device, group=None):
    """Decode this rank's share of an independent-block frame on `device`.

    Returns (d_out uint8 tensor, (lo, hi) block range, out_lens list).  The
    output stays resident on the rank's GPU (slots of block_max bytes).
    Raises the reference exception (via the exact path) if any rank found
    a bad block; linked frames raise ValueError (they do not shard)."""
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
    if k:
        d_in = torch.frombuffer(bytearray(frame[b0:b1]), dtype=torch.uint8).to(device)
        d_desc = torch.frombuffer(bytearray(bytes(local)[:k * ctypes.sizeof(lz4ada.BlockDesc)]),
                                  dtype=torch.uint8).to(device)
        d_st = torch.zeros(k * ctypes.sizeof(lz4ada.BlockStatus), dtype=torch.uint8,
                           device=device)
        stream = torch.cuda.current_stream(device)
        lz4ada.decode_blocks_device(d_in.data_ptr(), b1 - b0, d_desc.data_ptr(), k,
                                    d_out.data_ptr(), d_st.data_ptr(), stream.cuda_stream)
        stream.synchronize()
        raw = d_st.cpu().numpy().tobytes()
        sts = (lz4ada.BlockStatus * k).from_buffer_copy(raw)
        if block_errors([local[j] for j in range(k)], sts):
            status = SHARD_BLOCK_ERROR
        out_lens = [s.out_len for s in sts]
    if reduce_status(status, group, device) != SHARD_OK:
        lz4ada.decode_frame(frame)  # raises the reference exception
        # the exact path accepted it: a block reaches before its own start
        # (B.Indep set but ignored by the reference) -> linked data
        raise ValueError("frame has cross-block references (D2); decode it on one GPU "
                         "with lz4ada.decode_frame")
    return d_out, (lo, hi), out_lens
