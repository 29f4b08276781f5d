# Stored blocks hashed by the copying wave: parity tests, then the stored
# class with and without block checksums and the mixed headline decode
# (no regression).  Every step time-limited.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/st_$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  timeout -k 10 200 python tools/time_decode.py --kind stored --variant product --steps 10 2>&1 | grep -v amdgpu
  timeout -k 10 200 python tools/time_decode.py --kind stored --variant product --steps 10 --no-bcksum 2>&1 | grep -v amdgpu
  timeout -k 10 200 python tools/time_decode.py --kind mixed --variant product --steps 10 2>&1 | grep -v amdgpu
done
