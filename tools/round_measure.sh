# round-end measurement on the GPU box: the default bench line, then the same
# command under rocprofv3 --kernel-trace --stats (every step time-limited)
set -e
TAG=${1:-r03e}
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log
PMC_GROUPS=/dev/null bash tools/profile.sh $TAG
python tools/trace_by_grid.py gpurun_out/prof_$TAG/trace > gpurun_out/kernel_by_grid_$TAG.csv
