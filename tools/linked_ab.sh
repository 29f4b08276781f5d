#!/bin/bash
# configs[4] linked row, product vs variant builds (bo-lz4-ada_amd/_variants/*.so named
# in VARIANTS), on the GPU box: the row's wall time (tools/linked_time.py) alternated
# twice, then one rocprofv3 --kernel-trace --stats run each with the per-kernel
# averages of the linked path's kernels.  Usage: VARIANTS="oldjump" bash tools/linked_ab.sh [kinds]
KINDS=${1:-"mixed dense"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
libs=("")
for v in $VARIANTS; do libs+=("$R/bo-lz4-ada_amd/_variants/liblz4ada_hip_$v.so"); done
for k in $KINDS; do
  for rep in 1 2; do
    for lib in "${libs[@]}"; do
      name=$(basename "${lib:-product}" .so)
      echo -n "$name $k: "
      LZ4ADA_LIB=$lib timeout -k 10 200 python tools/linked_time.py $k 2>/dev/null || exit 1
    done
  done
  for lib in "${libs[@]}"; do
    name=$(basename "${lib:-product}" .so)
    out=$R/gpurun_out/lab/${name}_$k
    mkdir -p $out
    (cd /tmp && export TMPDIR=/tmp && LZ4ADA_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats \
       --output-format csv -d $out -o run -- python3 $R/tools/linked_time.py $k > $out/log 2>&1) || exit 1
    python3 - "$out" "$name" "$k" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
parts = []
for r in csv.DictReader(open(f)):
    n = r["Name"].split("(")[0].split("::")[-1].replace("void ", "")
    if n.startswith("k_"):
        parts.append(f"{n} {float(r['AverageNs']) / 1e3:.1f}us x{r['Calls']}")
print(sys.argv[2], sys.argv[3], " | ".join(sorted(parts)))
PY
  done
done
