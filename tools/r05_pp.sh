#!/bin/bash
# Round 5: k_decode_pp parity (focused) + timing against the one-wave kernel.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "pp" --timeout 120 --timeout-method thread > gpurun_out/r05_pp_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r05_pp_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/time_decode.py --kind mixed --variant idx1,pp,product --check && \
LZ4ADA_IDX_WAVES=p timeout -k 10 200 python tools/time_decode.py --kind mixed --variant product --check && \
timeout -k 10 200 python tools/time_decode.py --kind dense --variant idx1,pp --check && \
timeout -k 10 200 python tools/time_decode.py --kind mixed --blocks 1024 --variant idx1,idx2,pp && \
timeout -k 10 200 python tools/time_decode.py --kind mixed --blocks 8192 --unique 16 --variant idx1,pp
