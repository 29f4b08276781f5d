#!/bin/bash
# PMC passes over tools/wg_bench.py (k_decode_wg alone).  Usage: tools/wg_pmc.sh <tag> [args]
set -u
TAG=$1; shift
OUT=gpurun_out/wgpmc_$TAG
mkdir -p $OUT
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $line --kernel-trace --output-format csv -d $OUT/pmc$i -o run -- python3 tools/wg_bench.py "$@" > $OUT/pmc$i.log 2>&1 || exit 1
done < tools/pmc_groups.txt
echo done
