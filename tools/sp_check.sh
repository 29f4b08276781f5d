# sparse decoder: parity tests, then the literal class timed (golden-checked once)
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sparse.py > gpurun_out/sp_test.log 2>&1
timeout -k 10 200 python tools/time_decode.py --kind literal --variant idx_sparse,product --check > gpurun_out/sp_time.log 2>&1
