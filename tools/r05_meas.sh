#!/bin/bash
# Round 5 measurement: HBM-gather counts (diagnostic build), then the
# default bench line (c3 shares, facade row).  Every step time-limited.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/gathers.py --kinds mixed,dense > gpurun_out/r05b_gathers.txt 2>&1 || { tail -5 gpurun_out/r05b_gathers.txt; exit 1; }
cat gpurun_out/r05b_gathers.txt | grep -v amdgpu.ids
timeout -k 10 900 python bench.py > gpurun_out/r05b_bench.json 2> gpurun_out/r05b_bench.log || { tail -20 gpurun_out/r05b_bench.log; exit 1; }
cat gpurun_out/r05b_bench.json
