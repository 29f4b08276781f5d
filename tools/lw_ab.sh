#!/bin/bash
# Lone-decoder window A/B on the facade's 64 KiB frames (default windows vs a
# forced LZ4ADA_LONE_LW), then the lone and facade parity tests under the
# forced size (a size lone_window accepts: 512 ... 4096, or one a variant
# build adds).   bash tools/lw_ab.sh TAG LW
set -o pipefail
TAG=$1; LW=$2
O=gpurun_out; mkdir -p $O
out=$O/${TAG}_lw_ab.txt
: > $out
for indep in 1 0; do
  timeout -k 10 200 python tools/facade_time.py --indep $indep --kind $([ $indep = 1 ] && echo mixed || echo mixed_nod1) --block-max 65536 --blocks 64 --feed 4096 --reps 1 \
    --dump $O/${TAG}_f$indep.lz4 > $O/${TAG}_dump$indep.log 2>&1 || { echo "dump failed"; tail -15 $O/${TAG}_dump$indep.log; exit 1; }
  for rep in 1 2; do
    for lw in default $LW; do
      echo "== indep=$indep LW=$lw" >> $out
      if [ $lw = default ]; then
        timeout -k 10 120 bo-lz4-ada_amd/facade_bench $O/${TAG}_f$indep.lz4 4096 7 >> $out 2>&1 || exit 1
      else
        LZ4ADA_LONE_LW=$lw timeout -k 10 120 bo-lz4-ada_amd/facade_bench $O/${TAG}_f$indep.lz4 4096 7 >> $out 2>&1 || exit 1
      fi
    done
  done
  rm -f $O/${TAG}_f$indep.lz4 $O/${TAG}_f$indep.lz4.out
done
cat $out
LZ4ADA_LONE_LW=$LW timeout -k 10 600 python -u -m pytest tests/test_gpu_lone.py tests/test_gpu_facade.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $O/${TAG}_lw_tests.log 2>&1
rc=$?
tail -3 $O/${TAG}_lw_tests.log
exit $rc
