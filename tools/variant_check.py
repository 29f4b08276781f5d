#!/usr/bin/env python3
"""Decoder-variant check on the bench workload: for each class, run the
selected variants, count declined blocks (status DS_RETRY when run alone),
check every decoded slot against the generator's XXH32, and time K launches
with HIP events.

    python tools/variant_check.py --kinds mixed,dense --variants pc,idx,idx_alone
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

VARIANTS = {"pc": lz4ada.DECODE_PC,
            "idx": lz4ada.DECODE_IDX, "idx_alone": lz4ada.DECODE_IDX_ALONE}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", default="mixed")
    ap.add_argument("--variants", default="pc,idx")
    ap.add_argument("--blocks", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    bmax = 4 << 20
    for kind in args.kinds.split(","):
        recs = bench.make_unique_blocks(lz4ada.GEN_KINDS[kind], 64, bmax)
        d_frame, frame_len, d_desc, exp_hash, comp, raw, _ = bench.build_shard(
            recs, 0, args.blocks, bmax, dev)
        d_out = torch.empty(args.blocks * bmax, dtype=torch.uint8, device=dev)
        d_status = torch.zeros(args.blocks * 32, dtype=torch.uint8, device=dev)
        d_hash = torch.zeros(args.blocks, dtype=torch.int32, device=dev)
        sh = torch.cuda.current_stream(dev).cuda_stream
        for vname in args.variants.split(","):
            v = VARIANTS[vname]

            def launch():
                lz4ada.launch_decode_variant(d_frame.data_ptr(), frame_len, d_desc.data_ptr(),
                                             args.blocks, d_out.data_ptr(), d_status.data_ptr(),
                                             v, sh)
            d_out.fill_(0xAA)
            d_status.zero_()
            launch()
            torch.cuda.synchronize()
            st = bench.check_statuses(d_status, args.blocks)
            retry = sum(1 for s in st if s.code == lz4ada.DS_RETRY)
            other = sum(1 for s in st if s.code not in (0, lz4ada.DS_RETRY))
            lz4ada.output_checksums_device(d_out.data_ptr(), d_desc.data_ptr(), d_status.data_ptr(),
                                           args.blocks, d_hash.data_ptr(), sh)
            torch.cuda.synchronize()
            hs = d_hash.cpu().tolist()
            wrong = sum(1 for i, s in enumerate(st)
                        if s.code == 0 and (hs[i] & 0xFFFFFFFF) != exp_hash[i])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.steps):
                launch()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.steps
            print(f"{kind:8s} {vname:10s} {ms:9.3f} ms {(comp + raw) / ms / 1e6:8.1f} GB/s alg "
                  f"retry={retry} other={other} wrong={wrong}", flush=True)
        del d_frame, d_out


if __name__ == "__main__":
    main()
