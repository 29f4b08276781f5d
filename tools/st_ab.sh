# Stored-class A/B: product vs each bo-lz4-ada_amd/_variants/*.so, twice, with
# and without block checksums (GPU box).
set -e
for r in 1 2; do
  for lib in "" bo-lz4-ada_amd/_variants/liblz4ada_hip_stnt*.so; do
    LZ4ADA_LIB=$lib timeout -k 10 200 python tools/time_decode.py --kind stored --variant product --steps 10 --no-bcksum --check 2>/dev/null
    LZ4ADA_LIB=$lib timeout -k 10 200 python tools/time_decode.py --kind stored --variant product --steps 10 2>/dev/null
  done
done
