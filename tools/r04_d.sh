# round 4: full GPU suite + smoke, then the facade traces and the linked row A/B
set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/d_gpu.log 2>&1 || { tail -40 gpurun_out/d_gpu.log; exit 1; }
tail -1 gpurun_out/d_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v Warn | tail -1
for d in 0 1; do
  LZ4ADA_LINKED_DENSE=$d LZ4ADA_TRACE_LINKED=1 timeout -k 10 200 python tools/linked_time.py mixed > gpurun_out/d_link$d.log 2>&1 || { tail -20 gpurun_out/d_link$d.log; exit 1; }
  grep -v amdgpu gpurun_out/d_link$d.log | sort | uniq -c | sort -rn | head -8
done
LZ4ADA_TRACE_FACADE=1 timeout -k 10 200 python tools/facade_time.py --indep 1 --block-max 65536 --blocks 8 --feed 4096 --reps 1 > gpurun_out/d_fac64.log 2>&1 || true
LZ4ADA_TRACE_FACADE=1 timeout -k 10 200 python tools/facade_time.py --indep 0 --block-max 262144 --blocks 8 --feed 4096 --reps 1 > gpurun_out/d_facl.log 2>&1 || true
for f in "--indep 1 --block-max 65536 --blocks 256" "--indep 0 --block-max 262144 --blocks 64" "--indep 0 --block-max 65536 --blocks 256 --ccksum 0"; do
  timeout -k 10 200 python tools/facade_time.py $f --feed 4096 2>&1 | grep -v amdgpu
  LZ4ADA_FACADE_DECODER=pc timeout -k 10 200 python tools/facade_time.py $f --feed 4096 2>&1 | grep -v amdgpu
done
timeout -k 10 200 python tools/facade_time.py --indep 0 --block-max 65536 --blocks 256 --ccksum 0 --feed 0 2>&1 | grep -v amdgpu
