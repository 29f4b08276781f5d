#!/usr/bin/env python3
"""Summarise tools/pmc_real.sh into profiles/pmc_real.json: per real-data
class, k_decode_idx's HBM bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE,
MI355X_MICROARCH.md's gfx950 correction, separate passes) beside the
algorithmic bytes of the same launch; bench.py's real rows report it when
the kernel's code hash still matches.

    python tools/pmc_real_summary.py gpurun_out/prof_real"""
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import kernel_code_hash  # noqa: E402


def counter(d, name):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "k_decode_idx" in r["Kernel_Name"] and "k_decode_idx_" not in r["Kernel_Name"] \
                        and r["Counter_Name"] == name:
                    vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None


def main():
    src = sys.argv[1]
    out = {"kernel": "k_decode_idx", "kernel_code_sha16": kernel_code_hash("k_decode_idx"),
           "source": "tools/pmc_real.sh + tools/pmc_real_summary.py", "classes": {}}
    for t in sorted(glob.glob(os.path.join(src, "*_time.txt"))):
        cls = os.path.basename(t)[:-len("_time.txt")]
        line = open(t).read().strip().splitlines()[-1]
        m = re.search(r"([\d.]+) ms\s+([\d.]+) GB/s", line)
        ms, gbs = float(m.group(1)), float(m.group(2))
        alg = gbs * 1e9 * ms * 1e-3
        f, w = counter(os.path.join(src, cls + "_FETCH_SIZE"), "FETCH_SIZE"), \
            counter(os.path.join(src, cls + "_WRITE_SIZE"), "WRITE_SIZE")
        e = {"decoder_alone_ms": ms, "alg_bytes_per_launch": round(alg)}
        if f is not None and w is not None:
            hbm = f * 1024 * 2 + w * 1024
            e.update({"fetch_bytes_x2": round(f * 2048), "write_bytes": round(w * 1024),
                      "hbm_bytes_per_launch": round(hbm), "traffic_over_alg": round(hbm / alg, 2)})
        out["classes"][cls] = e
    path = os.path.join(ROOT, "profiles", "pmc_real.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
