# round-4 measurement: the default bench line; the same command under
# --kernel-trace --stats; PMC passes of the headline workload; a kernel trace
# of the facade on a linked frame at 4 KiB reads.  Every step time-limited.
set -e
TAG=${1:-r04a}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $line --kernel-trace --output-format csv -d $OUT/pmc$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-c3 --no-linked --no-64k --no-cpu-baseline --no-e2e --classes "" > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done < $GRAFT_REPO_ROOT/tools/pmc_groups.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/facade -o run -- python3 $GRAFT_REPO_ROOT/tools/facade_time.py --indep 0 --block-max 262144 --blocks 32 --feed 4096 --reps 1 > $OUT/facade.log 2>&1 || { echo "facade trace failed"; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/pmc_summary.py gpurun_out/prof_$TAG $TAG --first 7 > gpurun_out/pmcsum_$TAG.txt && python3 tools/trace_by_grid.py gpurun_out/prof_$TAG/trace > gpurun_out/kernel_by_grid_$TAG.csv
head -c 800 gpurun_out/bench_$TAG.json
