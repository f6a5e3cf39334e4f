#!/bin/bash
# bench lines at the other BASELINE configs (c2: 256^2 x 64 R=4; c4: 512^2 x 1024 R=16)
mkdir -p gpurun_out
for c in c2 c4; do
  timeout -k 10 300 python bench.py --config $c --cpu-baseline 0 > gpurun_out/cfg_$c.log 2>&1 || exit $?
  tail -1 gpurun_out/cfg_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', round(d['value']), 'grad-steps/s', d['kernels'], d['roofline']['frac'], d['quality'])"
done
