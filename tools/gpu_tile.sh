#!/bin/bash
# bench at C-pass tiles 1024 / 512 (fused S+C kernel), short runs
mkdir -p gpurun_out
for t in 1024 512 256; do
  QSC_CTILE=$t timeout -k 10 200 python bench.py --cpu-baseline 0 > gpurun_out/tile_$t.log 2>&1 || exit $?
  echo "tile $t: $(tail -1 gpurun_out/tile_$t.log | grep -o '"value": [0-9.]*')"
done
