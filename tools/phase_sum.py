#!/usr/bin/env python3
"""Summary of tools/phase_pmc.sh: per library, the decoder kernels' SQ
instruction counts per sequence and the deltas to the product build.
    python tools/phase_sum.py gpurun_out/phase_TAG [sequences]"""
import csv, glob, os, sys, collections
d = sys.argv[1]
NSEQ = float(sys.argv[2]) if len(sys.argv) > 2 else 268.4e6
rows = {}
for sub in sorted(glob.glob(d + "/*/")):
    name = os.path.basename(sub.rstrip("/")).replace("liblz4ada_hip_", "")
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    ids = collections.defaultdict(set)
    for f in glob.glob(sub + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("::")[-1]
            if not k.startswith(("k_decode", "k_index")):
                continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            ids[k].add(r["Dispatch_Id"])
    for k, cs in acc.items():
        n = len(ids[k])
        rows[(name, k)] = {c: v / n for c, v in cs.items()}
keys = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS"]
base = rows.get(("product", "k_decode_idx"))
print(f"{'lib':14s} {'kernel':14s} {'tot/seq':>8s} {'valu':>6s} {'salu':>6s} {'br':>6s} {'lds':>6s} {'Δtot':>7s} {'cyc/wave M':>10s} {'wait':>5s}")
for (name, k), cs in sorted(rows.items()):
    tot = sum(cs.get(c, 0) for c in keys)
    per = [cs.get(c, 0) / NSEQ for c in keys]
    dt = ""
    if base and k == "k_decode_idx":
        dt = "%+.2f" % ((tot - sum(base.get(c, 0) for c in keys)) / NSEQ)
    wc = cs.get("SQ_WAVE_CYCLES", 0) / max(cs.get("SQ_WAVES", 1), 1) / 1e6
    wf = cs.get("SQ_WAIT_ANY", 0) / max(cs.get("SQ_WAVE_CYCLES", 1), 1)
    print(f"{name:14s} {k:14s} {tot / NSEQ:8.2f} " + " ".join(f"{x:6.2f}" for x in per) + f" {dt:>7s} {wc:10.2f} {wf:5.2f}")
