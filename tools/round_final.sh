# full GPU suite, smoke(), then the round measurement (bench line + kernel trace)
set -e
TAG=${1:-r03f}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_full_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_full_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_full_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
bash tools/round_measure.sh $TAG
