# Round-4 check of the whole tree: XXH32 instruction costs, the full GPU
# test suite, smoke(), the default bench line.  Every step time-limited.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/full_$1
mkdir -p $O
timeout -k 10 60 ./tools/xxh_latency | tee $O/xxh_latency.txt
timeout -k 10 900 python -u -m pytest tests/ -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | grep -v amdgpu | tail -2
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline']['traffic_source']); print('linked', d['linked_c5']['decode_ms'])"
