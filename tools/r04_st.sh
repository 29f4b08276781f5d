# Same-box A/B of the stored-block checksum: the product (k_xxh32_rows
# beside the decoder's copy) against _variants/liblz4ada_hip_fusedst.so
# (the copying wave hashes the block, commit eee6b35), on the stored class
# with and without block checksums and on the mixed headline decode (the
# variant's k_decode_idx holds 211 VGPRs instead of 185).  Every step
# time-limited.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/st_$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for lib in "" bo-lz4-ada_amd/_variants/liblz4ada_hip_fusedst.so; do
    echo "== ${lib:-product}"
    LZ4ADA_LIB=$lib timeout -k 10 200 python tools/time_decode.py --kind mixed --variant product --steps 10 2>&1 | grep -v amdgpu
    LZ4ADA_LIB=$lib timeout -k 10 200 python tools/time_decode.py --kind stored --variant product --steps 10 2>&1 | grep -v amdgpu
  done
done
