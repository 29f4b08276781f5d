#!/usr/bin/env python3
"""Per-dispatch counter totals of a tools/pmc_split.sh run (sums over the
counter's dimensions), one line per kernel launch and counter above 1e5.

    python tools/pmc_dispatch.py gpurun_out/prof_TAG
"""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    for p in sorted(glob.glob(os.path.join(root, "p*"))):
        per, names = collections.defaultdict(float), {}
        for r in csv.DictReader(open(os.path.join(p, "run_counter_collection.csv"))):
            key = (int(r["Dispatch_Id"]), r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[key[0]] = r["Kernel_Name"].split("(")[0]
        for (d, c), v in sorted(per.items()):
            if v > 1e5 and "lz4ada" in names[d]:
                print(f"{os.path.basename(p)} {d:3d} {names[d]:28s} {c:26s} {v:.4g}")


if __name__ == "__main__":
    main()
