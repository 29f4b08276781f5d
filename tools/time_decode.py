#!/usr/bin/env python3
"""Decode-kernel timing for A/B experiments (no output check, so it also
times deliberately wrong experiment builds): the bench workload of one
class, K timed launches of the decoder selected by LZ4ADA_DECODER from the
library in LZ4ADA_LIB (default: the product).

    LZ4ADA_LIB=bo-lz4-ada_amd/_variants/liblz4ada_hip_x.so \
        python tools/time_decode.py --kind mixed
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import lz4ada  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="mixed")
    ap.add_argument("--blocks", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--checksums", action="store_true",
                    help="also run the block and output XXH32 kernels each step (and check them once)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    bmax = 4 << 20
    recs = bench.make_unique_blocks(lz4ada.GEN_KINDS[args.kind], 64, bmax)
    d_frame, frame_len, d_desc, exp_hash, comp, raw, descs = bench.build_shard(recs, 0, args.blocks,
                                                                                bmax, dev)
    d_out = torch.empty(args.blocks * bmax, dtype=torch.uint8, device=dev)
    d_status = torch.zeros(args.blocks * 32, dtype=torch.uint8, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    d_hash = torch.zeros(args.blocks, dtype=torch.int32, device=dev)

    def launch():
        if args.checksums:
            lz4ada.launch_block_checksums(d_frame.data_ptr(), d_desc.data_ptr(), args.blocks,
                                          d_status.data_ptr(), sh)
        lz4ada.launch_decode(d_frame.data_ptr(), frame_len, d_desc.data_ptr(), args.blocks,
                             d_out.data_ptr(), d_status.data_ptr(), sh)
        if args.checksums:
            lz4ada.output_checksums_device(d_out.data_ptr(), d_desc.data_ptr(), d_status.data_ptr(),
                                           args.blocks, d_hash.data_ptr(), sh)

    launch()
    torch.cuda.synchronize()
    if args.checksums:
        st = bench.check_statuses(d_status, args.blocks)
        assert all(s.cksum == d.cksum for s, d in zip(st, descs)), "block checksum mismatch"
        assert [h & 0xffffffff for h in d_hash.cpu().tolist()] == exp_hash, "output hash mismatch"
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.steps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    lib = os.path.basename(os.environ.get("LZ4ADA_LIB") or "product")
    print(f"{lib} {args.kind} {ms:.3f} ms  {(comp + raw) / ms / 1e6:.1f} GB/s alg")


if __name__ == "__main__":
    main()
