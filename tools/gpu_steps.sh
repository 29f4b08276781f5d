#!/bin/bash
# The GPU-box measurement steps in one parametrised script (it replaces the
# round-4 one-off tools/r04_*.sh; their results are in profiles/r04*):
#
#   bash tools/gpu_steps.sh TAG step [step ...]
#
#   suite    full `pytest -m gpu` (per-test timeout)
#   bench    the default bench line                  -> gpurun_out/TAG_bench.json
#   trace    rocprofv3 --kernel-trace --stats of the reduced bench (headline only)
#   pmc      one rocprofv3 --pmc pass per tools/pmc_groups.txt line, same command
#            (both into gpurun_out/prof_TAG/, as tools/pmc_summary.py reads them)
#   facade   bo-lz4-ada_amd/facade_bench on 64 KiB / 256 KiB linked / 4 MiB frames, 4 KiB reads,
#            with the facade's per-step laps (LZ4ADA_TRACE_FACADE) of the 64 KiB frame
#   lone     tools/lone_time.py over block sizes and classes
#   linked   tools/linked_time.py (configs[4]: mixed, dense, chain; then the mixed phases)
#   classes  tools/time_decode.py per content class (decoder alone and product step)
#   pp2      the pipelined two-wave decoder: its parity tests, then timed beside
#            k_decode_idx at 1,024 and 2,048 blocks
#   gathers  tools/gathers.py (needs the LZ4ADA_IDX_GATHERS variant build)
#
# Every step runs under its own time limit; the first failure ends the run.
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
REDUCED="--no-cpu-baseline --no-e2e --no-linked --no-64k --no-c3 --no-facade --classes= --real="
fail() { echo "step $1 failed"; tail -20 "$2" 2>/dev/null; exit 1; }
for step in "$@"; do
  case $step in
  suite)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > $O/${TAG}_suite.log 2>&1 || fail suite $O/${TAG}_suite.log
    tail -2 $O/${TAG}_suite.log ;;
  bench)
    timeout -k 10 900 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.log || fail bench $O/${TAG}_bench.log
    cat $O/${TAG}_bench.json ;;
  trace)
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
       -d $O/prof_${TAG}/trace -o run -- python3 $R/bench.py $REDUCED > $O/${TAG}_trace.log 2>&1) || fail trace $O/${TAG}_trace.log
    python3 tools/trace_by_grid.py $O/prof_${TAG}/trace > $O/${TAG}_kernel_by_grid.csv && head -12 $O/${TAG}_kernel_by_grid.csv ;;
  pmc)
    i=0
    while read -r grp; do
      [ -z "$grp" ] && continue
      i=$((i+1))
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
         -d $O/prof_${TAG}/pmc$i -o run -- python3 $R/bench.py $REDUCED > $O/${TAG}_pmc$i.log 2>&1) || fail pmc$i $O/${TAG}_pmc$i.log
    done < tools/pmc_groups.txt
    echo "pmc: $i passes (summary: python tools/pmc_summary.py gpurun_out/prof_${TAG} ${TAG})" ;;
  facade)
    timeout -k 10 400 python -c "import json, bench; print(json.dumps(bench.bench_facade()))" \
      > $O/${TAG}_facade.json 2> $O/${TAG}_facade.log || fail facade $O/${TAG}_facade.log
    cat $O/${TAG}_facade.json
    timeout -k 10 200 python tools/facade_time.py --indep 1 --block-max 65536 --blocks 64 --feed 4096 --reps 1 \
      --dump $O/${TAG}_f.lz4 > /dev/null 2>&1 || fail facade-dump /dev/null
    LZ4ADA_TRACE_FACADE=1 timeout -k 10 200 bo-lz4-ada_amd/facade_bench $O/${TAG}_f.lz4 4096 3 > $O/${TAG}_laps.log 2>&1 || fail laps $O/${TAG}_laps.log
    grep "lone " $O/${TAG}_laps.log | awk '{s[$3]+=$4; n[$3]++} END {for (k in s) printf "%-8s %.4f ms avg over %d\n", k, s[k]/n[k], n[k]}'
    rm -f $O/${TAG}_f.lz4 $O/${TAG}_f.lz4.out ;;
  lone)
    timeout -k 10 400 python tools/lone_time.py > $O/${TAG}_lone.txt 2>&1 || fail lone $O/${TAG}_lone.txt
    grep -v amdgpu $O/${TAG}_lone.txt ;;
  linked)
    for k in mixed dense chain; do
      timeout -k 10 300 python tools/linked_time.py $k >> $O/${TAG}_linked.txt 2>&1 || fail linked $O/${TAG}_linked.txt
    done
    LZ4ADA_TRACE_LINKED=1 timeout -k 10 300 python tools/linked_time.py mixed > $O/${TAG}_linked_phases.txt 2>&1 \
      || fail linked-phases $O/${TAG}_linked_phases.txt
    grep -v amdgpu $O/${TAG}_linked.txt
    tail -14 $O/${TAG}_linked_phases.txt ;;
  classes)
    for k in mixed dense literal rle; do
      timeout -k 10 200 python tools/time_decode.py --kind $k --variant idx1,product 2>&1 | grep -v amdgpu || fail classes /dev/null
    done ;;
  pp2)
    timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
      -k "pp2" > $O/${TAG}_pp2tests.log 2>&1 || fail pp2-tests $O/${TAG}_pp2tests.log
    tail -2 $O/${TAG}_pp2tests.log
    for k in mixed dense; do for nb in 1024 2048; do
      timeout -k 10 200 python tools/time_decode.py --kind $k --blocks $nb --variant pp2,idx1 --check 2>&1 \
        | grep -v amdgpu || fail pp2-time /dev/null
    done; done ;;
  gathers)
    timeout -k 10 300 python tools/gathers.py --kinds mixed,dense 2>&1 | grep -v amdgpu || fail gathers /dev/null ;;
  *)
    echo "unknown step $step"; exit 2 ;;
  esac
done
