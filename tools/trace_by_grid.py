#!/usr/bin/env python3
"""Per-kernel, per-grid-size dispatch averages from a rocprofv3
--kernel-trace run (the default bench launches k_decode_idx for three
workloads: the 2048-block roofline frame, configs[1]'s 16384 x 64 KiB blocks
and the linked configs[4] row, so the --stats average mixes them).

    python tools/trace_by_grid.py gpurun_out/prof_r02h_full/trace > profiles/r02h_kernel_by_grid.csv
"""
import collections
import csv
import glob
import sys


def main():
    f = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].split("::")[-1]
        wg = int(r["Workgroup_Size_X"])
        acc[(name, int(r["Grid_Size_X"]) // max(wg, 1), wg)].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "workgroups", "workgroup_size", "calls", "avg_ms", "min_ms", "max_ms"])
    for (name, g, wg), v in sorted(acc.items()):
        w.writerow([name, g, wg, len(v), f"{sum(v) / len(v):.4f}", f"{min(v):.4f}", f"{max(v):.4f}"])


if __name__ == "__main__":
    main()
