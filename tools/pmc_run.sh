#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, kernel trace only) of one
# command: tools/pmc_run.sh OUTDIR -- python3 tools/time_decode.py ...
# Groups from tools/pmc_groups.txt; summaries via tools/pmc_quick.py.
set -u
out=$1; shift; shift
cd /tmp && export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o p -- "$@" > "$out.p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done < "${PMC_GROUPS:-$GRAFT_REPO_ROOT/tools/pmc_groups.txt}"
python3 "$GRAFT_REPO_ROOT/tools/pmc_quick.py" "$out"
