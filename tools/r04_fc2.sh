# Facade from C: a context per frame vs one context for 8 frames (exact-path
# block counts), plus LZ4ADA_TRACE_FACADE phases of the one-context run.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/fc2_$1
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_linked.py tests/test_gpu_facade.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in "--indep 1 --block-max 4194304 --blocks 8" "--indep 0 --block-max 262144 --blocks 32"; do
  timeout -k 10 200 python tools/facade_time.py $cfg --feed 4096 --reps 1 --dump $O/frame.lz4 2>&1 | grep -v amdgpu
  timeout -k 10 200 ./tools/facade_c $O/frame.lz4 4096 3
  LZ4ADA_TRACE_FACADE=1 timeout -k 10 200 ./tools/facade_c $O/frame.lz4 4096 1 > $O/trace.log 2>&1
  grep "facade\]" $O/trace.log | awk '{print $2}' | sort | uniq -c
done
rm -f $O/frame.lz4 $O/frame.lz4.out
