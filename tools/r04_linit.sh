# Branch-free k_link_init: linked / narrow / facade tests, then configs[4]'s
# row with phase times (mixed, dense, chain).  Every step time-limited.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/linit_$1
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_linked.py tests/test_gpu_narrow.py tests/test_gpu_facade.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for k in mixed dense chain; do
    LZ4ADA_TRACE_LINKED=1 timeout -k 10 200 python tools/linked_time.py $k > $O/lt.log 2>&1
    grep -v amdgpu $O/lt.log | grep -E "init|jumps|decode_ms" | tail -3
  done
done
