#!/bin/bash
# A/B: default build vs variant libraries (bench value, fused kernel time, C-finish time),
# alternating, REPS rounds:  REPS=3 bash tools/gpu_ab.sh variants/libqsc_a.so variants/libqsc_b.so
mkdir -p gpurun_out
for rep in $(seq ${REPS:-3}); do
  for lib in default "$@"; do
    if [ $lib = default ]; then
      timeout -k 10 200 python bench.py --cpu-baseline 0 ${BENCH_ARGS} > gpurun_out/ab.log 2>&1 || exit $?
    else
      QSC_LIB_PATH=$lib timeout -k 10 200 python bench.py --cpu-baseline 0 ${BENCH_ARGS} > gpurun_out/ab.log 2>&1 || exit $?
    fi
    tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%-32s' % '$lib', round(d['value']), round(d['kernels']['scfused_us'] or 0, 2), round(d['kernels']['cfinish_us'], 2))"
  done
done
