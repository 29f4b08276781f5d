set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sparse.py > gpurun_out/sp_test.log 2>&1; tail -1 gpurun_out/sp_test.log
for k in mixed dense rle; do
for v in "" base; do
  lib=""; [ -n "$v" ] && lib=bo-lz4-ada_amd/_variants/liblz4ada_hip_$v.so
  LZ4ADA_LIB=$lib timeout -k 10 200 python tools/time_decode.py --kind $k --variant product --steps 10 2>/dev/null
done; done
