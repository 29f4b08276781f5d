#!/bin/bash
# k_decode_pc (LZ4ADA_DECODER=pc) timing of the product and every variant (GPU box).
shopt -s nullglob
for lib in "" bo-lz4-ada_amd/_variants/*.so; do
  LZ4ADA_DECODER=pc LZ4ADA_LIB=$lib timeout -k 10 200 python3 tools/time_decode.py --kind mixed --blocks 512 || exit 1
done
