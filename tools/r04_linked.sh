# Linked frames after the in-place byte writes (no emit pass): GPU tests of
# the linked, narrow and facade paths, then configs[4]'s row with phase
# times and a kernel trace.  Every step time-limited.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/linked_$1
mkdir -p $O
timeout -k 10 60 ./tools/xxh_latency | tee $O/xxh_latency.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_linked.py tests/test_gpu_narrow.py tests/test_gpu_facade.py tests/test_gpu_lone.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for f in 1 0 1; do
for k in mixed dense chain; do
  echo "== LZ4ADA_LINK_FWD=$f $k"
  LZ4ADA_LINK_FWD=$f LZ4ADA_TRACE_LINKED=1 timeout -k 10 200 python tools/linked_time.py $k > $O/lt_$k.log 2>&1
  grep -v amdgpu $O/lt_$k.log | tail -12
done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/linked_time.py mixed > $GRAFT_REPO_ROOT/$O/trace.log 2>&1
cd $GRAFT_REPO_ROOT && python3 tools/trace_by_grid.py $O/trace | grep -E "link|decode_idx|k_index"
