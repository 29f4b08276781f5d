#!/bin/bash
# Per-kernel A/B: rocprofv3 --kernel-trace --stats of tools/time_decode.py for
# the product and every bo-lz4-ada_amd/_variants/*.so; prints the average
# duration of each decode kernel.  Usage (GPU box): [EXTRA=--checksums] bash tools/ab_prof.sh [kinds]
KINDS=${1:-"mixed dense"}
shopt -s nullglob
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for k in $KINDS; do
  for lib in "" bo-lz4-ada_amd/_variants/*.so; do
    name=$(basename "${lib:-product}" .so)
    out=gpurun_out/abp/${name}_$k
    mkdir -p $out
    LZ4ADA_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run \
      -- python3 tools/time_decode.py --kind $k $EXTRA > $out/log 2>&1 || exit 1
    python3 - "$out" "$name" "$k" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
parts = []
for r in csv.DictReader(open(f)):
    n = r["Name"].split("(")[0].split("::")[-1]
    if n.startswith("k_"):
        parts.append(f"{n} {float(r['AverageNs']) / 1e6:.3f}")
print(sys.argv[2], sys.argv[3], " | ".join(sorted(parts)))
PY
  done
done
