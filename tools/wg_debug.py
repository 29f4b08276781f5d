#!/usr/bin/env python3
"""Run the workgroup decoder alone on bench blocks with a diagnostic build.

    make -C bo-lz4-ada_amd/csrc wgcheck
    python tools/wg_debug.py --kind mixed --blocks 16 [--lib wgcheck]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("--kind", default="mixed")
ap.add_argument("--blocks", type=int, default=16)
ap.add_argument("--first", type=int, default=0)
ap.add_argument("--bmax", type=int, default=4 << 20)
ap.add_argument("--lib", default="wgcheck")
args = ap.parse_args()
if args.lib:
    os.environ["LZ4ADA_LIB"] = os.path.join(ROOT, "bo-lz4-ada_amd", f"liblz4ada_hip_{args.lib}.so")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))
import torch  # noqa: E402
import lz4ada  # noqa: E402
import lz4frame  # noqa: E402

blocks = [lz4ada.gen_block(lz4ada.GEN_KINDS[args.kind], 0x4C5A3441 + i, args.bmax)
          for i in range(args.first, args.first + args.blocks)]
frame, raw = lz4frame.build_frame([(c, r, False) for c, r in blocks], args.bmax)
info, descs = lz4ada.frame_index(frame)
nb = info.nblocks
dev = torch.device("cuda:0")
d_frame = torch.frombuffer(bytearray(frame), dtype=torch.uint8).to(dev)
d_desc = torch.frombuffer(bytearray(bytes(descs)[:nb * 32]), dtype=torch.uint8).to(dev)
d_out = torch.zeros(nb * args.bmax, dtype=torch.uint8, device=dev)
d_st = torch.zeros(nb * 32, dtype=torch.uint8, device=dev)
lz4ada.launch_decode_wg(d_frame.data_ptr(), len(frame), d_desc.data_ptr(), nb, d_out.data_ptr(),
                        d_st.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
st = (lz4ada.BlockStatus * nb).from_buffer_copy(d_st.cpu().numpy().tobytes())
out = d_out.cpu().numpy().tobytes()
for i, (c, r) in enumerate(blocks):
    got = out[i * args.bmax:i * args.bmax + len(r)]
    j = next((k for k in range(len(r)) if got[k] != r[k]), -1)
    print(f"block {args.first + i}: code={st[i].code} out_len={st[i].out_len} want={len(r)} "
          f"comp={len(c)} first_diff={j}", flush=True)
