# stored copies: NT (no block checksums) / cached (with) vs all-plain (stnt0), then PC sampling of the headline decoder
set -e
for r in 1 2; do
  for lib in "" bo-lz4-ada_amd/_variants/liblz4ada_hip_stnt0.so; do
    LZ4ADA_LIB=$lib timeout -k 10 200 python tools/time_decode.py --kind stored --variant product --steps 10 --no-bcksum --check 2>&1 | grep -v amdgpu
    LZ4ADA_LIB=$lib timeout -k 10 200 python tools/time_decode.py --kind stored --variant product --steps 10 2>&1 | grep -v amdgpu
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 10 --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pcs -o pcs -- python3 $GRAFT_REPO_ROOT/tools/time_decode.py --kind mixed --blocks 1024 --steps 2 --variant idx1 > $GRAFT_REPO_ROOT/gpurun_out/pcs.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/pcs.log; exit 1; }
ls -la $GRAFT_REPO_ROOT/gpurun_out/pcs/* | head
