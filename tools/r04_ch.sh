# k_lone_chain walking only the first wrong run: lone + facade parity tests,
# lone decode at 512 / 1024-byte windows, the facade laps at the default
# windows and at 512 (where round 4's serial walk cost 24 us per block).
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lone.py tests/test_gpu_facade.py > gpurun_out/ch_tests.log 2>&1 || { tail -30 gpurun_out/ch_tests.log; exit 1; }
tail -1 gpurun_out/ch_tests.log
timeout -k 10 300 env LZ4ADA_LONE_LW=512 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lone.py > gpurun_out/ch_tests512.log 2>&1 || { tail -30 gpurun_out/ch_tests512.log; exit 1; }
tail -1 gpurun_out/ch_tests512.log
for lw in 512 1024; do
  echo "== LZ4ADA_LONE_LW=$lw"
  for sz in 65536 262144 524288 1048576 4194304; do
    LZ4ADA_LONE_LW=$lw timeout -k 10 120 python tools/lone_time.py --size $sz --reps 50 --kinds mixed,dense,literal 2>&1 | grep -v amdgpu
  done
done
echo "== facade default windows"
bash tools/r04_ftr.sh ch3
echo "== facade LZ4ADA_LONE_LW=512"
LZ4ADA_LONE_LW=512 bash tools/r04_ftr.sh ch4
