#!/usr/bin/env python3
"""CPU model of k_decode_idx's batch structure on generator blocks: batch
cut (128 sequences / 4,080 output bytes), match classes (HBM / ring), and
the ring pieces' dependency steps (ring_pieces: 64-piece chunks, a piece
waits for lower pieces of its chunk that write its source range).
    python tools/ring_sim.py [kind] [blocks]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bo-lz4-ada_amd"))
import lz4ada  # noqa: E402

def seqs(comp):
    out, p, o, n = [], 0, 0, len(comp)
    while p < n:
        t = comp[p]; p += 1
        L = t >> 4
        if L == 15:
            while True:
                e = comp[p]; p += 1; L += e
                if e != 255: break
        lit = p; p += L
        if p >= n:
            out.append((o, L, 0, 0)); break
        off = comp[p] | (comp[p + 1] << 8); p += 2
        M = t & 15
        if M == 15:
            while True:
                e = comp[p]; p += 1; M += e
                if e != 255: break
        out.append((o, L, off, M + 4)); o += L + M + 4
    return out

def pattern_step(off):
    return off * (16 // off) if off <= 8 else off

def pieces_of(m, off, ml):
    if off < 16 and off < ml:
        st = pattern_step(off)
        return [(m + k * st, min(16, ml - k * st), m - off, m) for k in range((ml + st - 1) // st)]
    wide = ml > off
    res = []
    for k in range((ml + 15) // 16):
        pd = m + 16 * k; pn = min(16, ml - 16 * k)
        if wide: res.append((pd, pn, m - off, m))
        else: res.append((pd, pn, m - off + 16 * k, m - off + 16 * k + pn))
    return res

def chunk_steps(pcs):
    # pcs: list of (pd, pn, slo, shi) in output order; returns dependency steps
    depth = []
    for i, (pd, pn, slo, shi) in enumerate(pcs):
        d = 0
        for j in range(i):
            qd, qn = pcs[j][0], pcs[j][1]
            if qd < shi and qd + qn > slo:
                d = max(d, depth[j])
        depth.append(d + 1)
    return max(depth) if depth else 0

def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "mixed"
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    st = {"batches": 0, "seq": 0, "hbm": 0, "ring": 0, "near": 0, "ownlit": 0, "steps": 0, "chunks": 0,
          "ring_batches": 0, "pieces": 0, "lit_pieces": 0, "hbm_pieces": 0, "fwd_steps": 0}
    for b in range(nb):
        comp, raw = lz4ada.gen_block(lz4ada.GEN_KINDS[kind], 1000 + b, 4 << 20)
        S = seqs(comp)
        i = 0
        while i < len(S):
            o_b = S[i][0]
            j = i; tot = 0
            while j < len(S) and j - i < 128 and tot + S[j][1] + S[j][3] <= 4080:
                tot += S[j][1] + S[j][3]; j += 1
            if j == i: j = i + 1
            B = S[i:j]; i = j
            st["batches"] += 1; st["seq"] += len(B)
            glo = o_b - 4080 - 16
            ring = []
            fwd = []
            for (d, L, off, ml) in B:
                st["lit_pieces"] += (L + 15) // 16
                if ml == 0: continue
                m = d + L
                if m - off < glo:
                    st["hbm"] += 1; st["hbm_pieces"] += (ml + 15) // 16; continue
                st["ring"] += 1
                if m - off + min(off, ml) > o_b: st["near"] += 1
                if off <= L: st["ownlit"] += 1
                pcs = pieces_of(m, off, ml)
                ring.append(pcs)
                # forwarding model: a match whose source lies in its own literals
                # (off <= L) or before the batch has no dependency
                fwd.append([] if (off <= L or m - off + min(off, ml) <= o_b) else pcs)
            if any(ml > 32 for (_, _, off, ml) in B if ml):
                pass
            allp = [p for m in ring for p in m]
            st["pieces"] += len(allp)
            if allp: st["ring_batches"] += 1
            for c in range(0, len(allp), 64):
                st["chunks"] += 1
                st["steps"] += chunk_steps(allp[c:c + 64])
            fp = [p for m in fwd for p in m]
            nf = len([m for m in ring]) - len([m for m in fwd if m])
            for c in range(0, len(fp), 64):
                st["fwd_steps"] += chunk_steps(fp[c:c + 64])
            # the forwarded ones (independent) cost one step per 64-piece chunk
            nind = sum(len(m) for m, f in zip(ring, fwd) if not f)
            st["fwd_steps"] += (nind + 63) // 64
    nb_ = st["batches"]
    print(kind, {k: (round(v / nb_, 2) if k not in ("batches",) else v) for k, v in st.items()})
    print("per seq: seq/batch %.1f  ring steps/batch %.2f  fwd model %.2f" % (st["seq"] / nb_, st["steps"] / nb_, st["fwd_steps"] / nb_))

main()
