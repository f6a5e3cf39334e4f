#!/bin/bash
# GPU tests, then the C3 bench (no CPU leg) under each environment setting in $ENVS
# (space-separated VAR=VALUE items, "-" for none):  OUT=x ENVS="- QSC_SIGNED_ROWS=0" bash tools/gpu_ab_env.sh
G=gpurun_out/${OUT:-ab}
mkdir -p $G
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $G/pytest_gpu.log 2>&1; rc=$?
  tail -3 $G/pytest_gpu.log
  faulted $G/pytest_gpu.log && { echo FAULT; exit 99; }
  [ $rc -ne 0 ] && { grep -E "FAILED|Error" $G/pytest_gpu.log | head; exit $rc; }
fi
i=0
for rep in ${REPS:-1}; do
for e in ${ENVS:--}; do
  i=$((i+1))
  if [ "$e" = "-" ]; then ev=""; else ev="${e//,/ }"; fi
  env $ev timeout -k 10 300 python bench.py --cpu-baseline 0 ${BENCH_ARGS} > $G/bench_$i.log 2>&1 || { tail -5 $G/bench_$i.log; exit 1; }
  tail -1 $G/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$e', round(d['value']), {x: round(v, 2) for x, v in k.items() if x.endswith('_us') and v})"
done
done
