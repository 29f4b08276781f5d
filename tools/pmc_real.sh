#!/bin/bash
# HBM traffic of k_decode_idx on the real-data classes:
# one rocprofv3 --pmc pass per counter (FETCH_SIZE, WRITE_SIZE: the guide's
# separate passes), tools/time_decode.py --real NAME --variant idx1, 2,048
# blocks; then  python tools/pmc_real_summary.py gpurun_out/prof_real
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_real
mkdir -p $O
for cls in ${1:-t1111k liblz4_text}; do
  timeout -k 10 200 python3 $R/tools/time_decode.py --real $cls --variant idx1 --steps 3 > $O/${cls}_time.txt 2>/dev/null || exit 1
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace --output-format csv \
       -d $O/${cls}_$c -o run -- python3 $R/tools/time_decode.py --real $cls --variant idx1 --steps 3 > $O/${cls}_$c.log 2>&1) || exit 1
  done
done
cat $O/*_time.txt
