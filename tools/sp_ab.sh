# literal-heavy decoder: parity, product step and decoder alone (vs the scalar-parse build)
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sparse.py > gpurun_out/sp_test.log 2>&1 ; tail -1 gpurun_out/sp_test.log
for v in "" spsalu spscal; do
  lib=""; [ -n "$v" ] && lib=bo-lz4-ada_amd/_variants/liblz4ada_hip_$v.so
  LZ4ADA_LIB=$lib timeout -k 10 200 python tools/time_decode.py --kind literal --variant idx_sparse,product 2>/dev/null
done
