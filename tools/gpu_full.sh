set -e
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_full.log 2>&1 || { tail -30 gpurun_out/gpu_full.log; exit 1; }
tail -2 gpurun_out/gpu_full.log
timeout -k 10 200 python tools/time_decode.py --kind literal --variant idx_sparse,product --check 2>/dev/null
