# round 4: full GPU suite, then the default bench line (each step time-limited)
set -e
TAG=${1:-r04a}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_$TAG.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
cat gpurun_out/bench_$TAG.json | head -c 600
