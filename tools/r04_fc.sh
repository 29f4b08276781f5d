# The facade from C (tools/facade_c) against the Python loop
# (tools/facade_time.py) on the same frames, 4 KiB reads.  Every step
# time-limited.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/fc_$1
mkdir -p $O
for cfg in "--indep 1 --block-max 65536 --blocks 64" "--indep 0 --block-max 262144 --blocks 32" "--indep 0 --block-max 65536 --blocks 64 --kind mixed_nod1" "--indep 1 --block-max 4194304 --blocks 8"; do
  timeout -k 10 200 python tools/facade_time.py $cfg --feed 4096 --reps 5 --dump $O/frame.lz4 2>&1 | grep -v amdgpu
  timeout -k 10 200 ./tools/facade_c $O/frame.lz4 4096 5
done
rm -f $O/frame.lz4 $O/frame.lz4.out
