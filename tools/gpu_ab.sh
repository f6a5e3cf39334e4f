#!/bin/bash
# A/B: default build vs a variant library (bench value + fused kernel time), alternating
mkdir -p gpurun_out
V=${1:-variants/libqsc_noprio.so}
for rep in 1 2 3; do
  for lib in default $V; do
    if [ $lib = default ]; then
      timeout -k 10 200 python bench.py --cpu-baseline 0 > gpurun_out/ab.log 2>&1 || exit $?
    else
      QSC_LIB_PATH=$lib timeout -k 10 200 python bench.py --cpu-baseline 0 > gpurun_out/ab.log 2>&1 || exit $?
    fi
    tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['value']), round(d['kernels']['scfused_us'] or 0, 2), round(d['kernels']['cfinish_us'], 2))"
  done
done
