# Same-box A/B: k_xxh32_rows loads in flight (XW 48 product, 32, 24) on the
# mixed headline step (checksums overlapped with the decode) and on the
# stored class with block checksums.  Every step time-limited.
set -e
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for lib in "" bo-lz4-ada_amd/_variants/liblz4ada_hip_xw32.so bo-lz4-ada_amd/_variants/liblz4ada_hip_xw24.so; do
    echo "== ${lib:-product}"
    LZ4ADA_LIB=$lib timeout -k 10 200 python tools/time_decode.py --kind mixed --variant product --steps 10 2>&1 | grep -v amdgpu
    LZ4ADA_LIB=$lib timeout -k 10 200 python tools/time_decode.py --kind stored --variant product --steps 10 2>&1 | grep -v amdgpu
  done
done
