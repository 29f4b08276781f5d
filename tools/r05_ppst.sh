#!/bin/bash
# Round 5: k_decode_pp phase stamps; the one-wave kernel at 64-sequence batches.
set -o pipefail
timeout -k 10 200 python tools/pp_stamps.py --kinds mixed,dense && \
timeout -k 10 200 python tools/pp_stamps.py --kinds mixed --blocks 1024 && \
LZ4ADA_LIB=bo-lz4-ada_amd/_variants/liblz4ada_hip_seq64.so timeout -k 10 200 python tools/time_decode.py --kind mixed --variant idx1 && \
LZ4ADA_LIB=bo-lz4-ada_amd/_variants/liblz4ada_hip_seq64.so timeout -k 10 200 python tools/time_decode.py --kind mixed --blocks 1024 --variant idx1 && \
LZ4ADA_LIB=bo-lz4-ada_amd/_variants/liblz4ada_hip_seq64.so timeout -k 10 200 python tools/time_decode.py --kind dense --variant idx1
