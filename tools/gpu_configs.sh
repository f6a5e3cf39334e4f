#!/bin/bash
# bench lines at the other BASELINE configs (c2: 256^2 x 64 R=4; c4: 512^2 x 1024 R=16, per-GPU
# K-slab share and the whole map on one GPU), stopping at the first failure
mkdir -p gpurun_out/cfg
run() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py --cpu-baseline 0 "$@" > gpurun_out/cfg/$tag.log 2>&1 || exit $?
  tail -1 gpurun_out/cfg/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), 'grad-steps/s', d['config'].get('workload'), d['roofline']['frac'])"
}
run c2 --config c2
run c4 --config c4
run c4_strong --config c4 --scaling strong
