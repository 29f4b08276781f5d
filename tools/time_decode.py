#!/usr/bin/env python3
"""Decode-kernel timing for A/B experiments (no output check unless
--check, so it also times deliberately wrong experiment builds): the bench
workload of one class, K timed launches of one decoder variant from the
library in LZ4ADA_LIB (default: the product).

    LZ4ADA_LIB=bo-lz4-ada_amd/_variants/liblz4ada_hip_x.so \
        python tools/time_decode.py --kind mixed --variant idx
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))

import torch  # noqa: E402
import xxhash  # noqa: E402

import bench  # noqa: E402
import lz4ada  # noqa: E402
import lz4frame  # noqa: E402

VARIANTS = {"pc": lz4ada.DECODE_PC,
            "idx": lz4ada.DECODE_IDX, "idx_alone": lz4ada.DECODE_IDX_ALONE,
            "idx_sparse": lz4ada.DECODE_IDX_SPARSE,
            "idx1": lz4ada.DECODE_IDX1_ALONE,
            "pp2": lz4ada.DECODE_PP2_ALONE, "split": lz4ada.DECODE_IDX_SPLIT}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="mixed")
    ap.add_argument("--real", default="", help="t1111k / liblz4_text: encoder blocks (bench.real_sources)")
    ap.add_argument("--blocks", type=int, default=2048)
    ap.add_argument("--unique", type=int, default=16)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--variant", default="idx", help=",".join(VARIANTS) + ",product")
    ap.add_argument("--no-bcksum", action="store_true")
    ap.add_argument("--check", action="store_true", help="golden-check the output once")
    ap.add_argument("--block-max", type=int, default=4 << 20)
    ap.add_argument("--slot-pad", type=int, default=0, help="bytes between output slots (layout experiment)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    bmax = args.block_max
    M = (lz4ada, lz4frame, xxhash, torch)
    if args.real:
        recs = bench.real_sources(args.real)[0]
        args.kind = args.real
    else:
        recs = bench.make_unique_blocks(lz4ada, lz4frame, xxhash, args.kind, args.unique, bmax,
                                        block_cksum=not args.no_bcksum)
    d_frame, frame_len, d_desc, exp_hash, comp, raw, descs = bench.assemble_shard(
        lz4ada, torch, recs, 0, args.blocks, bmax, dev, slot_pad=args.slot_pad)
    d_out = torch.empty(args.blocks * (bmax + args.slot_pad), dtype=torch.uint8, device=dev)
    d_status = torch.zeros(args.blocks * 32, dtype=torch.uint8, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    d_hash = torch.zeros(args.blocks, dtype=torch.int32, device=dev)
    fp, dp, op, sp = d_frame.data_ptr(), d_desc.data_ptr(), d_out.data_ptr(), d_status.data_ptr()

    for name in args.variant.split(","):
        def launch():
            if name == "product":
                lz4ada.decode_blocks_device(fp, frame_len, dp, args.blocks, op, sp, sh)
            elif name == "cksum":
                lz4ada.launch_block_checksums(fp, dp, args.blocks, sp, sh)
            else:
                lz4ada.launch_decode_variant(fp, frame_len, dp, args.blocks, op, sp, VARIANTS[name],
                                             sh)

        d_status.zero_()
        launch()
        torch.cuda.synchronize()
        st = bench.check_statuses(lz4ada, d_status, args.blocks)
        codes = {}
        for s in st:
            codes[s.code] = codes.get(s.code, 0) + 1
        if args.check and name == "cksum":
            bad = [i for i in range(args.blocks) if st[i].cksum != descs[i].cksum]
            assert not bad, f"block checksum mismatch {bad[:5]}"
        elif args.check:
            if name != "product":
                lz4ada.launch_block_checksums(fp, dp, args.blocks, sp, sh)
            bench.golden_check(lz4ada, torch, d_status, descs, args.blocks, op, dp, sp, d_hash,
                               exp_hash, sh, name)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            launch()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.steps
        lib = os.path.basename(os.environ.get("LZ4ADA_LIB") or "product")
        print(f"{lib} {args.kind} {name}: {ms:.3f} ms  {(comp + raw) / ms / 1e6:.1f} GB/s alg "
              f"frac {(comp + raw) / ms / 1e6 / 8000:.4f}  codes {codes}", flush=True)


if __name__ == "__main__":
    main()
