# A/B of the literal-heavy decoder's variant builds (timing only; EXP builds give wrong output)
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sparse.py 2>&1 | tail -2
for v in "" spnocopy; do
  lib=""; [ -n "$v" ] && lib=bo-lz4-ada_amd/_variants/liblz4ada_hip_$v.so
  LZ4ADA_LIB=$lib timeout -k 10 200 python tools/time_decode.py --kind literal --variant idx_sparse,product 2>/dev/null
done
timeout -k 10 200 python tools/sp_stamps.py 2>/dev/null
