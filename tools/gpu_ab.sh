#!/bin/bash
# A/B (ENVS entries: comma-separated VAR=value sets): default build vs variant libraries (bench value, us/step, fused kernel and C-finish time),
# alternating, REPS rounds:  REPS=3 [ENVS="QSC_FIN=0 QSC_FIN=1"] bash tools/gpu_ab.sh variants/libqsc_a.so ...
mkdir -p gpurun_out
for rep in $(seq ${REPS:-3}); do
  for e in ${ENVS:-QSC_FIN=0}; do
    for lib in default "$@"; do
      if [ $lib = default ]; then lp=""; else lp="QSC_LIB_PATH=$lib"; fi
      env ${e//,/ } $lp timeout -k 10 200 python bench.py --cpu-baseline 0 ${BENCH_ARGS} > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
      tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('%-10s %-32s' % ('$e', '$lib'), round(d['value']), round(d['ms_per_step']*1e3, 2), 'us/step', {x: round(v, 2) for x, v in k.items() if x.endswith('_us') and v})"
    done
  done
done
