#!/bin/bash
# One GPU step for a decoder change: golden-checked timing (decoder alone,
# mixed and dense), the instruction counts of the headline kernel
# (SQ_INSTS_*, one --pmc pass), then the index-decoder parity tests.
#   bash tools/quick_ab.sh TAG [pytest -k expression]
set -o pipefail
TAG=$1; KEXPR=${2:-"idx or bench_blocks"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab_${TAG}
mkdir -p $O
for k in mixed dense; do
  timeout -k 10 200 python tools/time_decode.py --kind $k --variant idx1 --check 2>&1 | grep -v amdgpu | tee -a $O/time.txt \
    || { echo "time $k failed"; exit 1; }
done
CTR="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES"
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace --output-format csv \
   -d $O/pmc/product -o run -- python3 $R/tools/time_decode.py --kind mixed --variant idx1 --steps 2 > $O/pmc.log 2>&1) \
   || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
python3 tools/phase_sum.py $O/pmc | tee $O/pmc_sum.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "$KEXPR" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
exit $rc
