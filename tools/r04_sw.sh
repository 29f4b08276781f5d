# Window sweep under the first-run chain walk: forced 512 - 4096-byte
# windows, 64 KiB - 4 MiB blocks, lone decoder only; the lone tests at 2048.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 env LZ4ADA_LONE_LW=2048 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lone.py > gpurun_out/sw_tests.log 2>&1 || { tail -30 gpurun_out/sw_tests.log; exit 1; }
tail -1 gpurun_out/sw_tests.log
for lw in 512 1024 2048 4096; do
  echo "== LZ4ADA_LONE_LW=$lw"
  for sz in 65536 131072 262144 524288 1048576 2097152 4194304; do
    LZ4ADA_LONE_LW=$lw timeout -k 10 120 python tools/lone_time.py --size $sz --reps 30 --kinds mixed,dense,literal 2>&1 | grep -v amdgpu
  done
done
