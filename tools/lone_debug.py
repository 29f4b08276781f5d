"""Diagnostics for the lone-block decoder: the control record and the
window entries against the true chain (from a Python parse of the block)."""
import ctypes
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import lz4ada  # noqa: E402
import torch  # noqa: E402
from _lz4build import encode, sparse_seqs  # noqa: E402

LW = 4096


def chain(comp):
    p, n, starts = 0, len(comp), []
    while p < n:
        starts.append(p)
        t = comp[p]
        L, M, x = t >> 4, t & 15, p + 1
        if L == 15:
            while True:
                e = comp[x]; x += 1; L += e
                if e != 255:
                    break
        x += L
        if x >= n:
            break
        x += 2
        if M == 15:
            while True:
                e = comp[x]; x += 1
                if e != 255:
                    break
        p = x
    return starts


def main(seed):
    rng = random.Random(seed)
    seqs = sparse_seqs(rng, 3 << 20, lit_lo=1, lit_hi=20000,
                       offs=[1, 2, 3, 7, 16, 100, 5000, 60000], mls=[4, 18, 19, 300, 70000])
    comp, raw = encode(seqs, final_lits=rng.randbytes(rng.choice([0, 5, 40])))
    n, cap = len(comp), 4 << 20
    nwin = (n + LW - 1) // LW
    d_in = torch.frombuffer(bytearray(comp + b"\0" * 16), dtype=torch.uint8).cuda()
    d_out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    d_st = torch.zeros(32, dtype=torch.uint8, device="cuda")
    sb = lz4ada.lone_scratch_bytes(n, cap)
    d_sc = torch.zeros(sb, dtype=torch.uint8, device="cuda")
    lz4ada.launch_decode_lone(d_in.data_ptr(), n, d_out.data_ptr(), cap, d_st.data_ptr(),
                              d_sc.data_ptr(), sb, 0)
    torch.cuda.synchronize()
    sc = d_sc.cpu().numpy()
    base = d_sc.data_ptr()
    exit_tab = sc[:4 * n].view("<u4")
    entry = sc[12 * n:12 * n + 4 * (nwin + 1)].view("<u4")
    obase = sc[12 * n + 4 * (nwin + 1):12 * n + 8 * (nwin + 1)].view("<u4")
    ctl_off = ((base + 12 * n + 12 * (nwin + 1) + 63) & ~63) - base
    ctl = sc[ctl_off:ctl_off + 16].view("<u4")
    st = lz4ada.BlockStatus.from_buffer_copy(d_st.cpu().numpy().tobytes())
    print(f"seed {seed}: n={n} nwin={nwin} raw={len(raw)} status={st.code} out_len={st.out_len} "
          f"ctl code={ctl[0]} total={ctl[1]} iters={ctl[3]}")
    starts = chain(comp)
    ss = set(starts)
    # true entries
    import bisect
    bad = 0
    for w in range(nwin):
        i = bisect.bisect_left(starts, w * LW)
        te = starts[i] if i < len(starts) else n
        if te != entry[w]:
            bad += 1
            if bad < 5:
                print("  window", w, "entry", entry[w], "true", te)
    print("  entry mismatches:", bad)
    if st.code == 0:
        got = d_out[:st.out_len].cpu().numpy().tobytes()
        print("  bytes equal:", got == raw)


if __name__ == "__main__":
    for s in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
        main(s)
