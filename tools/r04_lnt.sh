# Linked frames with nontemporal streaming in k_link_init / k_link_jump:
# tests, then a same-box A/B against the cached build (_variants/linknt0)
# on configs[4]'s row with phase times.  Every step time-limited.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/lnt_$1
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_linked.py tests/test_gpu_facade.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for lib in "" bo-lz4-ada_amd/_variants/liblz4ada_hip_linknt0.so; do
    for k in mixed dense; do
      echo "== ${lib:-product} $k"
      LZ4ADA_LIB=$lib LZ4ADA_TRACE_LINKED=1 timeout -k 10 200 python tools/linked_time.py $k > $O/lt.log 2>&1
      grep -v amdgpu $O/lt.log | tail -6
    done
  done
done
