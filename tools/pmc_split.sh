#!/bin/bash
# Per-pass memory counters of the index decoder (diagnostic, round 5): the
# split variant (k_index, then k_decode_idx's pass 2, two launches) and the
# fused one, on one content class, one rocprofv3 --pmc pass per group.
#   [VARIANTS=split,idx1] [BLOCKS=2048] bash tools/pmc_split.sh TAG KIND "GROUP1" "GROUP2" ...
# -> gpurun_out/prof_TAG/pN/run_counter_collection.csv (tools/pmc_dispatch.py reads them)
set -o pipefail
TAG=$1; KIND=$2; shift 2
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
[ -n "$LZ4ADA_LIB" ] && export LZ4ADA_LIB=$(readlink -f "$LZ4ADA_LIB")  # (the runs start in /tmp)
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/prof_$TAG/p$i -o run \
    -- python3 $GRAFT_REPO_ROOT/tools/time_decode.py --kind $KIND --variant ${VARIANTS:-split,idx1} \
       --blocks ${BLOCKS:-2048} --steps 2 \
    > $O/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/${TAG}_p$i.log; exit 1; }
done
echo done
