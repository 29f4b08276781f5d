#!/bin/bash
# Round-5 probe: GPU suite, then decode timing of batch-cut variants (mixed,
# dense; 2048 and 1024 blocks; one- and two-wave index decoders).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_gpu.log 2>&1 || { tail -30 gpurun_out/r05_gpu.log; exit 1; }
tail -2 gpurun_out/r05_gpu.log
for k in mixed dense; do
  for nb in 2048 1024; do
    timeout -k 10 200 python tools/time_decode.py --kind $k --blocks $nb --variant idx1,idx2,cksum,product || exit 1
    for v in seq64 seq96; do
      LZ4ADA_LIB=bo-lz4-ada_amd/_variants/liblz4ada_hip_$v.so timeout -k 10 200 python tools/time_decode.py --kind $k --blocks $nb --variant idx1 || exit 1
    done
  done
done
