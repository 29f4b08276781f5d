#!/usr/bin/env python3
"""Per-kernel durations and the gaps before each kernel (start minus the
previous kernel's end on the same queue) from a rocprofv3 kernel trace of
the facade (tools/facade_trace.sh).

    python tools/facade_gaps.py gpurun_out/prof_TAG_facade
"""
import collections
import csv
import glob
import os
import sys


def main():
    rows = []
    for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur, gap = collections.defaultdict(list), collections.defaultdict(list)
    prev_end = None
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("lz4ada::", "")
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        dur[name].append((e - s) / 1e3)
        if prev_end is not None and 0 <= s - prev_end < 200e3:
            gap[name].append((s - prev_end) / 1e3)
        prev_end = e
    print(f"{'kernel':28s} {'calls':>6s} {'avg us':>8s} {'gap before us':>14s}")
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        g = gap[k]
        print(f"{k:28s} {len(dur[k]):6d} {sum(dur[k]) / len(dur[k]):8.2f} "
              f"{(sum(g) / len(g)) if g else float('nan'):14.2f}")


if __name__ == "__main__":
    main()
