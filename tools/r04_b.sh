# round 4 check: the new paths' parity first (two-wave decoder, facade, linked), then timings
set -e
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -k "idx_decoder_alone or bench_blocks or idx_decoder_on_vectors" --timeout 120 --timeout-method thread > gpurun_out/b_par.log 2>&1 || { tail -40 gpurun_out/b_par.log; exit 1; }
tail -1 gpurun_out/b_par.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_facade.py tests/test_gpu_linked.py -x -q --timeout 120 --timeout-method thread > gpurun_out/b_fac.log 2>&1 || { tail -40 gpurun_out/b_fac.log; exit 1; }
tail -1 gpurun_out/b_fac.log
for k in mixed dense; do
  timeout -k 10 150 python tools/time_decode.py --kind $k --variant idx1,idx2,product --check 2>&1 | grep -v Warn
  timeout -k 10 150 python tools/time_decode.py --kind $k --blocks 1024 --variant idx1,idx2 2>&1 | grep -v Warn
done
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --classes "" --no-c3 --no-64k --no-cpu-baseline --no-e2e > gpurun_out/b_bench.json 2> gpurun_out/b_bench.log || { tail -20 gpurun_out/b_bench.log; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/b_bench.json')); print(r['value'], r['ms_per_step'], r['roofline']['frac'], r['linked_c5']['decode_ms'], r['linked_c5']['frac'])"
