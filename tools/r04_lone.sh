# Lone-block decoder and the facade's lone path: GPU tests of the lone and
# facade paths, kernel latency by block size (adaptive window and forced
# LZ4ADA_LONE_LW), facade throughput on linked 256 KiB and independent 64 KiB
# blocks, and a per-phase trace of a few facade blocks.  Every step
# time-limited.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/lone_$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lone.py tests/test_gpu_facade.py tests/test_gpu_narrow.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for lw in "" 1024 2048 4096; do
  echo "== LZ4ADA_LONE_LW=${lw:-adaptive}"
  for sz in 16384 65536 262144 1048576 4194304; do
    LZ4ADA_LONE_LW=$lw timeout -k 10 120 python tools/lone_time.py --size $sz --reps 20 2>&1 | grep -v amdgpu
  done
done
echo "== facade"
for i in 1 2; do
timeout -k 10 200 python tools/facade_time.py --indep 0 --block-max 262144 --blocks 32 --feed 4096 --reps 5 2>&1 | grep -v amdgpu
timeout -k 10 200 python tools/facade_time.py --indep 1 --block-max 65536 --blocks 64 --feed 4096 --reps 5 2>&1 | grep -v amdgpu
timeout -k 10 200 python tools/facade_time.py --indep 0 --block-max 65536 --blocks 64 --feed 4096 --reps 5 --ccksum 0 2>&1 | grep -v amdgpu
timeout -k 10 200 python tools/facade_time.py --kind mixed_nod1 --indep 0 --block-max 65536 --blocks 64 --feed 4096 --reps 5 2>&1 | grep -v amdgpu
timeout -k 10 200 python tools/facade_time.py --indep 1 --block-max 4194304 --blocks 8 --feed 4096 --reps 3 2>&1 | grep -v amdgpu
done
LZ4ADA_TRACE_FACADE=1 timeout -k 10 200 python tools/facade_time.py --indep 0 --block-max 262144 --blocks 6 --feed 4096 --reps 1 > $O/trace.log 2>&1
grep facade $O/trace.log | tail -24
