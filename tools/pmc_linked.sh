#!/bin/bash
# HBM traffic of the configs[4] linked row's kernels (GPU box): two rocprofv3
# --pmc passes (FETCH_SIZE, then WRITE_SIZE: one pass cannot hold both) over
# tools/linked_time.py, each with --kernel-trace only, then the per-kernel
# average per dispatch (tools/pmc_dispatch.py layout: gpurun_out/prof_TAG/p1, p2).
#   bash tools/pmc_linked.sh TAG [kind]
TAG=$1
KIND=${2:-mixed}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace --output-format csv \
     -d $O/p$i -o run -- python3 $R/tools/linked_time.py $KIND > $O/p$i.log 2>&1) || { echo "pmc pass $c failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 - "$O" <<'PY'
import collections, csv, glob, os, sys
root = sys.argv[1]
tot = collections.defaultdict(lambda: [0.0, set()])
for p in sorted(glob.glob(os.path.join(root, "p*"))):
    f = glob.glob(os.path.join(p, "**", "run_counter_collection.csv"), recursive=True)
    if not f:
        continue
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1]
        if not k.startswith("k_"):
            continue
        t = tot[(k, r["Counter_Name"])]
        t[0] += float(r["Counter_Value"])
        t[1].add(int(r["Dispatch_Id"]))
for (k, c), (v, ds) in sorted(tot.items()):
    print(f"{k:24s} {c:12s} {v / len(ds):14.4g} per dispatch (raw counter, KB; before the guide's gfx950 corrections) over {len(ds)} dispatches")
PY
