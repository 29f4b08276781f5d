# Linked 64 KiB frames with quirk-D1 blocks through the bulk path: adaptive
# read-ahead batches (product) vs the 512 MiB batches before (cap0), plus the
# linked / facade GPU tests.  Every step time-limited.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/d1_$1
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_linked.py tests/test_gpu_facade.py tests/test_gpu_narrow.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for nb in 64 256; do
  for lib in "" bo-lz4-ada_amd/_variants/liblz4ada_hip_cap0.so; do
    LZ4ADA_LIB=$lib timeout -k 10 300 python tools/d1_frame_time.py $nb mixed 2>&1 | grep -v amdgpu
  done
done
