# Lone resolve slice sweep: forced 1024 / 2048 / 4096-word slices, lone
# decoder only, 64 KiB - 4 MiB blocks; then the lone parity tests at 1024.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 env LZ4ADA_LONE_SLICE=1024 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lone.py > gpurun_out/sl_tests.log 2>&1 && tail -1 gpurun_out/sl_tests.log
for sl in 4096 2048 1024 4096 1024; do
  echo "== LZ4ADA_LONE_SLICE=$sl"
  for sz in 65536 262144 1048576 4194304; do
    LZ4ADA_LONE_SLICE=$sl timeout -k 10 120 python tools/lone_time.py --size $sz --reps 50 --kinds mixed,dense,literal 2>&1 | grep -v amdgpu
  done
done
