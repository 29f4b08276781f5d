#!/usr/bin/env python3
"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv (one or
more pass directories): python tools/pmc_quick.py gpurun_out/pmcA gpurun_out/pmcB"""
import collections
import csv
import glob
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(set))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("::")[-1]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k][r["Counter_Name"]].add(r["Dispatch_Id"])
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        n = len(cnt[k][c])
        print(f"   {c:24s} {v / n:16.4g}  (per dispatch, {n} dispatches)")
