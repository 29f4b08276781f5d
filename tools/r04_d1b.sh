# Quirk D1 emulated in the lone decoder: facade / linked / lone / narrow GPU
# tests, then the D1 frame through the bulk path and the facade (64 KiB
# linked blocks, uniform offsets).  Every step time-limited.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/d1b_$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_facade.py tests/test_gpu_linked.py tests/test_gpu_lone.py tests/test_gpu_narrow.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for nb in 64 256; do
  timeout -k 10 300 python tools/d1_frame_time.py $nb mixed 2>&1 | grep -v amdgpu
done
timeout -k 10 200 python tools/facade_time.py --indep 0 --block-max 65536 --blocks 64 --feed 4096 --reps 5 --ccksum 0 2>&1 | grep -v amdgpu
timeout -k 10 200 python tools/facade_time.py --indep 0 --block-max 65536 --blocks 64 --feed 4096 --reps 5 --ccksum 0 --dump $O/f.lz4 2>&1 | grep -v amdgpu
timeout -k 10 200 ./tools/facade_c $O/f.lz4 4096 5
rm -f $O/f.lz4 $O/f.lz4.out
