# Per-step trace of the facade's lone path (LZ4ADA_TRACE_FACADE) from C on
# 64 KiB independent and 256 KiB linked blocks, and the kernel trace of the
# 64 KiB run.  Every step time-limited.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/ftr_$1
mkdir -p $O
for cfg in "--indep 1 --block-max 65536 --blocks 64" "--indep 0 --block-max 262144 --blocks 32"; do
  timeout -k 10 200 python tools/facade_time.py $cfg --feed 4096 --reps 1 --dump $O/f.lz4 2>&1 | grep -v amdgpu
  LZ4ADA_TRACE_FACADE=1 timeout -k 10 200 ./tools/facade_c $O/f.lz4 4096 3 > $O/t.log 2>&1
  grep "lone " $O/t.log | awk '{s[$3]+=$4; n[$3]++} END {for (k in s) printf "%-8s %.4f ms avg over %d\n", k, s[k]/n[k], n[k]}'
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o run -- $GRAFT_REPO_ROOT/tools/facade_c $GRAFT_REPO_ROOT/$O/f.lz4 4096 3 > $GRAFT_REPO_ROOT/$O/kt.log 2>&1
cd $GRAFT_REPO_ROOT && python3 tools/trace_by_grid.py $O/kt | grep -E "lone|copy|fill" | head -20
rm -f $O/f.lz4 $O/f.lz4.out
