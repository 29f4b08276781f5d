#!/bin/bash
# Kernel trace of the streaming facade on a frame of 64 x 64 KiB independent
# mixed blocks fed 4 KiB per Update call (bo-lz4-ada_amd/facade_bench):
# per-kernel durations and the gaps between one block's kernels.
#   bash tools/facade_trace.sh TAG  -> gpurun_out/TAG_facade_kernels.txt
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 200 python tools/facade_time.py --indep 1 --block-max 65536 --blocks 64 --feed 4096 --reps 1 \
  --dump $O/${TAG}_f.lz4 > /dev/null 2>&1 || { echo "dump failed"; exit 1; }
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
   -d $O/prof_${TAG}_facade -o run -- $R/bo-lz4-ada_amd/facade_bench $O/${TAG}_f.lz4 4096 3 \
   > $O/${TAG}_facade_trace.log 2>&1) || { echo "trace failed"; tail -5 $O/${TAG}_facade_trace.log; exit 1; }
python3 tools/facade_gaps.py $O/prof_${TAG}_facade > $O/${TAG}_facade_kernels.txt && cat $O/${TAG}_facade_kernels.txt
rm -f $O/${TAG}_f.lz4 $O/${TAG}_f.lz4.out
