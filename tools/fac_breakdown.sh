#!/bin/bash
# Streaming-facade timing breakdown (GPU box): 16 x 4 MiB mixed blocks through
# Init_With_Header + Update at several feed sizes, with and without the
# frame's block / content checksums (tools/facade_time.py).
set -e
mkdir -p gpurun_out
T="timeout -k 10 120 python tools/facade_time.py"
$T --feed 4096 > gpurun_out/fac.log 2>&1
$T --feed 4096 --bcksum 0 >> gpurun_out/fac.log 2>&1
$T --feed 4096 --bcksum 0 --ccksum 0 >> gpurun_out/fac.log 2>&1
$T --feed 65536 >> gpurun_out/fac.log 2>&1
$T --feed 0 >> gpurun_out/fac.log 2>&1
grep facade gpurun_out/fac.log
