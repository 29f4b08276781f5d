"""Device-to-device copy rate on this part, the ceiling the stored class is
priced against (stored note): torch's copy of
an 8 GiB buffer (the runtime's own copy kernel) and of 2048 x 4 MiB pieces
whose source starts 7 bytes past a 16-byte boundary (a stored block's
payload in a frame is not aligned).

    python tools/copy_ceiling.py
"""
import torch


def timed(fn, steps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(steps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps


def main():
    dev = torch.device("cuda:0")
    n = 8 << 30
    src = torch.randint(0, 255, (n + 4096,), dtype=torch.uint8, device=dev)
    dst = torch.empty(n, dtype=torch.uint8, device=dev)
    ms = timed(lambda: dst.copy_(src[:n]))
    print(f"aligned 8 GiB copy: {ms:.3f} ms  {2 * n / ms / 1e6:.1f} GB/s (read+write)")
    ms = timed(lambda: dst.copy_(src[7:n + 7]))
    print(f"+7-byte source 8 GiB copy: {ms:.3f} ms  {2 * n / ms / 1e6:.1f} GB/s (read+write)")
    s32, d32 = src[:n].view(torch.int32), dst.view(torch.int32)
    ms = timed(lambda: d32.copy_(s32))
    print(f"int32 view copy: {ms:.3f} ms  {2 * n / ms / 1e6:.1f} GB/s (read+write)")
    ms = timed(lambda: dst.fill_(3))
    print(f"8 GiB fill: {ms:.3f} ms  {n / ms / 1e6:.1f} GB/s (write)")
    ms = timed(lambda: src[:n].view(torch.int64).sum())
    print(f"8 GiB int64 sum: {ms:.3f} ms  {n / ms / 1e6:.1f} GB/s (read)")


if __name__ == "__main__":
    main()
