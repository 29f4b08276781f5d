#!/bin/bash
# Usage (on the GPU box): tools/profile.sh <tag> [bench args...]
# 1) kernel-trace + stats of the bench command, 2) one --pmc pass per
# counter group (groups may not mix with sys/runtime tracing on this pool).
set -u
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
ARGS="$@"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit 1
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $line --kernel-trace --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py $ARGS > $OUT/pmc$i.log 2>&1 || exit 1
done < tools/pmc_groups.txt
echo done
