#!/bin/bash
# Linked-row (configs[4]) and workgroup-decoder timing of the product and every
# variant in bo-lz4-ada_amd/_variants (GPU box).
shopt -s nullglob
for lib in "" bo-lz4-ada_amd/_variants/*.so; do
  LZ4ADA_DECODER=wg LZ4ADA_LIB=$lib timeout -k 10 200 python3 tools/time_decode.py --kind mixed --blocks 512 || exit 1
  LZ4ADA_LIB=$lib timeout -k 10 200 python3 - <<'PY' || exit 1
import os, sys
sys.path.insert(0, "."); sys.path.insert(0, "bo-lz4-ada_amd")
import torch, bench
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
r = bench.bench_linked(dev, stream.cuda_stream, stream)
print(os.path.basename(os.environ.get("LZ4ADA_LIB") or "product"), "linked", r["decode_ms"], "ms")
PY
done
