#!/bin/bash
# A/B decode timing of variant builds (make -C bo-lz4-ada_amd/csrc variant NAME=..):
#   bash tools/ab.sh [classes] -- times the decode kernel (tools/time_decode.py, no
#   output check) for the product and every bo-lz4-ada_amd/_variants/*.so; a
#   class real:NAME takes bench.real_sources' blocks
CLASSES=${1:-"mixed dense literal"}
shopt -s nullglob
for k in $CLASSES; do
  case $k in real:*) KARG="--real ${k#real:}";; *) KARG="--kind $k";; esac
  for lib in "" bo-lz4-ada_amd/_variants/*.so; do
    LZ4ADA_LIB=$lib timeout -k 10 200 python tools/time_decode.py $KARG 2>/dev/null || exit 1
  done
done
