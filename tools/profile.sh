#!/bin/bash
# Usage (on the GPU box): tools/profile.sh <tag> [bench args...]
# 1) kernel-trace + stats of the bench command, 2) one --pmc pass per
# counter group (groups may not mix with sys/runtime tracing on this pool).
# Every step has its own time limit; the first failure ends the script.
set -u
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py "$@" > $OUT/trace.log 2>&1 || { echo "trace failed"; exit 1; }
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $line --kernel-trace --output-format csv -d $OUT/pmc$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py "$@" > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done < ${PMC_GROUPS:-$GRAFT_REPO_ROOT/tools/pmc_groups.txt}
echo done
