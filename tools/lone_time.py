"""Lone-block latency: one 4 MiB block decoded by lz4ada_launch_decode_lone
(the whole GPU) against the workgroup decoder (the facade's round-2 choice),
per synthetic kind.  Output checked."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))
import lz4ada  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", default="mixed,dense,literal,rle")
    ap.add_argument("--size", type=int, default=4 << 20)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    stream = torch.cuda.current_stream()
    for kind in args.kinds.split(","):
        comp, raw = lz4ada.gen_block(lz4ada.GEN_KINDS[kind], 0x4C5A, args.size)
        n, cap = len(comp), args.size
        d_in = torch.frombuffer(bytearray(comp + b"\0" * 16), dtype=torch.uint8).cuda()
        d_out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
        d_st = torch.zeros(32, dtype=torch.uint8, device="cuda")
        sb = lz4ada.lone_scratch_bytes(n, cap)
        d_sc = torch.empty(sb, dtype=torch.uint8, device="cuda")
        desc = lz4ada.BlockDesc()
        desc.in_off, desc.in_len, desc.out_off, desc.out_cap = 0, n, 0, cap
        d_desc = torch.frombuffer(bytearray(bytes(desc)), dtype=torch.uint8).cuda()

        def lone():
            lz4ada.launch_decode_lone(d_in.data_ptr(), n, d_out.data_ptr(), cap, d_st.data_ptr(),
                                      d_sc.data_ptr(), sb, stream.cuda_stream)

        def pc():
            lz4ada.launch_decode_variant(d_in.data_ptr(), n, d_desc.data_ptr(), 1, d_out.data_ptr(),
                                         d_st.data_ptr(), lz4ada.DECODE_PC, stream.cuda_stream)

        res = {}
        for name, fn in (("lone", lone), ("pc", pc)):
            fn()
            torch.cuda.synchronize()
            st = lz4ada.BlockStatus.from_buffer_copy(d_st.cpu().numpy().tobytes())
            ok = st.code == 0 and d_out[:st.out_len].cpu().numpy().tobytes() == raw
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[name] = (e0.elapsed_time(e1) / args.reps, ok, st.code)
        print(f"{kind:8s} {args.size >> 10} KiB (comp {n}): lone {res['lone'][0]:.3f} ms "
              f"ok={res['lone'][1]}  pc {res['pc'][0]:.3f} ms ok={res['pc'][1]}", flush=True)


if __name__ == "__main__":
    main()
