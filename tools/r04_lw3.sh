# Lone decoder with the ratio-aware window rule: lone parity tests, the
# default choice at 64 KiB - 4 MiB, then the facade (64 KiB independent,
# 256 KiB linked) from Python and C.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lone.py tests/test_gpu_facade.py > gpurun_out/lw3_tests.log 2>&1 && tail -1 gpurun_out/lw3_tests.log
for sz in 65536 131072 262144 524288 1048576 2097152 4194304; do
  timeout -k 10 120 python tools/lone_time.py --size $sz --reps 50 --kinds mixed,dense,literal 2>&1 | grep -v amdgpu
done
bash tools/r04_ftr.sh d
