#!/bin/bash
# A/B decode timing of variant builds (make -C bo-lz4-ada_amd/csrc variant NAME=..):
#   bash tools/ab.sh [classes] -- runs bench.py per class for the product and every
#   bo-lz4-ada_amd/_variants/*.so, one line each: lib class MiB/s kernel_ms frac
CLASSES=${1:-"mixed dense literal"}
shopt -s nullglob
for lib in "" bo-lz4-ada_amd/_variants/*.so; do
  for k in $CLASSES; do
    LZ4ADA_LIB=$lib timeout -k 10 200 python bench.py --kind $k --no-cpu-baseline --no-e2e 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('${lib:-product}'.split('/')[-1], '$k', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" || exit 1
  done
done
