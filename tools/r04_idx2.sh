# two-wave index decoder: focused parity first, then timing against the one-wave kernel
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "idx_decoder_alone or bench_blocks or idx_decoder_on_vectors" --timeout 120 --timeout-method thread > gpurun_out/idx2_par.log 2>&1 || { tail -40 gpurun_out/idx2_par.log; exit 1; }
tail -2 gpurun_out/idx2_par.log
for k in mixed dense; do
  timeout -k 10 150 python tools/time_decode.py --kind $k --variant idx1,idx2,product --check 2>&1 | grep -v Warn
  timeout -k 10 150 python tools/time_decode.py --kind $k --blocks 1024 --variant idx1,idx2 2>&1 | grep -v Warn
done
