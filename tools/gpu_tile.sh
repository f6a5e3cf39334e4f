#!/bin/bash
# bench at C-pass tiles (fused S+C kernel), short runs without the CPU baseline
#   TILES="1024 512" bash tools/gpu_tile.sh
mkdir -p gpurun_out
for t in ${TILES:-1024 512 256}; do
  QSC_CTILE=$t timeout -k 10 200 python bench.py --cpu-baseline 0 ${BENCH_ARGS} > gpurun_out/tile_$t.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/tile_$t.log').read().strip().splitlines()[-1]);print('tile $t value',round(d['value']),'scfused_us',d['kernels']['scfused_us'],'cfinish_us',d['kernels']['cfinish_us'])"
done
