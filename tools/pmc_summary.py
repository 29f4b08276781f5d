#!/usr/bin/env python3
"""Summarise a tools/gpu_steps.sh pmc run (trace + one pass per counter group) into profiles/.

    python tools/pmc_summary.py gpurun_out/prof_r01 r01 [--kind mixed --blocks 2048]

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_pmc.json           per-kernel counters, averaged per dispatch
  profiles/pmc_decode.json          HBM bytes per decode launch (k_decode_pc, the default), read by bench.py

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3):
FETCH_SIZE and WRITE_SIZE are in KiB, collected in separate --pmc passes;
on gfx950 FETCH_SIZE reports half the bytes of 16-byte-per-lane streaming
reads, so it is doubled; WRITE_SIZE is exact for 16-byte-per-lane stores.
Both count L2 misses served by the Infinity Cache as well as HBM.
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import kernel_code_hash  # noqa: E402
KERNELS = ("k_decode_idx_zl", "k_decode_idx_lk", "k_decode_pp2", "k_decode_idx", "k_index", "k_decode_sparse", "k_decode_pc", "k_decode_blocks",
           "k_lone_windows", "k_lone_chain", "k_lone_words", "k_lone_resolve",
           "k_link_fill", "k_link_init", "k_link_jump", "k_link_tail",
           "k_xxh32_rows", "k_serial_block", "k_xxh32_update",
           "k_compact")


def short(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("tag")
    ap.add_argument("--kind", default="mixed")
    ap.add_argument("--blocks", type=int, default=2048)
    ap.add_argument("--block-max", type=int, default=4 << 20)
    ap.add_argument("--first", type=int, default=0,
                    help="only the first N dispatches of each kernel (the bench's headline "
                         "workload runs first: warmup + steps)")
    args = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)

    stats = os.path.join(args.dir, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, f"{args.tag}_kernel_stats.csv"))
    avg_ns = {}
    with open(stats) as fh:
        for r in csv.DictReader(fh):
            k = short(r["Name"])
            if k:
                avg_ns[k] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}

    # per-dispatch durations from the kernel trace (the --stats average mixes
    # every workload the command runs; --first keeps the headline's)
    trace = os.path.join(args.dir, "trace", "run_kernel_trace.csv")
    if args.first and os.path.exists(trace):
        durs = collections.defaultdict(list)
        with open(trace) as fh:
            rows = sorted(csv.DictReader(fh), key=lambda r: int(r["Dispatch_Id"]))
        for r in rows:
            k = short(r["Kernel_Name"])
            if k:
                durs[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for k, v in durs.items():
            v = v[:args.first]
            avg_ns[k] = {"calls": len(v), "avg_ns": sum(v) / len(v), "first_dispatches": args.first}
        # the headline's dispatches, one row each (the --stats average mixes workloads)
        with open(os.path.join(prof, f"{args.tag}_headline_dispatches.csv"), "w") as fh:
            fh.write("kernel,dispatch_index,duration_ns\n")
            for k, v in sorted(durs.items()):
                for i, ns in enumerate(v[:args.first]):
                    fh.write(f"{k},{i},{ns}\n")

    counters = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(args.dir, "pmc*", "run_counter_collection.csv"))):
        with open(f) as fh:
            rows = list(csv.DictReader(fh))
        seen = collections.defaultdict(list)  # kernel -> dispatch ids in order
        for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
            k = short(r["Kernel_Name"])
            if k and int(r["Dispatch_Id"]) not in seen[k]:
                seen[k].append(int(r["Dispatch_Id"]))
        for r in rows:
            k = short(r["Kernel_Name"])
            if k and (not args.first or int(r["Dispatch_Id"]) in seen[k][:args.first]):
                counters[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    per = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in counters.items()}

    out = {"tag": args.tag, "kernels": {}}
    for k in sorted(set(avg_ns) | set(per)):
        e = dict(avg_ns.get(k, {}))
        e["counters_per_dispatch"] = per.get(k, {})
        c = per.get(k, {})
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["fetch_bytes_raw"] = c["FETCH_SIZE"] * 1024
            e["fetch_bytes_x2"] = c["FETCH_SIZE"] * 1024 * 2
            e["write_bytes"] = c["WRITE_SIZE"] * 1024
            e["hbm_bytes_per_launch"] = e["fetch_bytes_x2"] + e["write_bytes"]
        if "SQ_WAVE_CYCLES" in c:
            wc = c["SQ_WAVE_CYCLES"]
            e["issue_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0) / wc
            e["wait_frac"] = c.get("SQ_WAIT_ANY", 0) / wc
        insts = sum(c.get(n, 0) for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
                                          "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                                          "SQ_INSTS_BRANCH"))
        if insts:
            e["wave_instructions"] = insts
        out["kernels"][k] = e
    with open(os.path.join(prof, f"{args.tag}_pmc.json"), "w") as fh:
        json.dump(out, fh, indent=1)

    ks = out["kernels"]
    if "k_decode_idx" in ks and "k_index" in ks and not args.first:
        # the default decode path is two kernels: report their sum per launch
        a, b = ks["k_index"], ks["k_decode_idx"]
        dname = "k_index+k_decode_idx"
        dec = {}
        for f in ("hbm_bytes_per_launch", "fetch_bytes_x2", "write_bytes", "avg_ns"):
            if f in a and f in b:
                dec[f] = a[f] + b[f]
    elif "k_decode_idx" in ks:
        # fused (k_decode_idx mode 3 runs pass 1 too): one kernel
        dname = "k_decode_idx"
        dec = ks[dname]
    else:
        dname = next((k for k in ("k_decode_pc", "k_decode_blocks") if k in ks), None)
        dec = ks.get(dname, {})
    if "hbm_bytes_per_launch" in dec:
        pj = {"config": {"kind": args.kind, "blocks": args.blocks, "block_max": args.block_max},
              "kernel": dname,
              "hbm_bytes_per_launch": round(dec["hbm_bytes_per_launch"]),
              "fetch_bytes_x2": round(dec["fetch_bytes_x2"]),
              "write_bytes": round(dec["write_bytes"]),
              "avg_ns": dec.get("avg_ns"),
              # bench.py reuses the figure only while the kernel's machine code matches
              "kernel_code_sha16": "+".join(str(kernel_code_hash(k)) for k in dname.split("+")),
              "source": f"profiles/{args.tag}_pmc.json (tools/gpu_steps.sh pmc + tools/pmc_summary.py)"}
        with open(os.path.join(prof, "pmc_decode.json"), "w") as fh:
            json.dump(pj, fh, indent=1)
    print(json.dumps({k: {kk: v for kk, v in e.items() if kk != "counters_per_dispatch"}
                      for k, e in out["kernels"].items()}, indent=1))


if __name__ == "__main__":
    main()
