#!/bin/bash
# Round-6 session i: fused launch S-step slices claimed from an LDS counter (QSC_DYN_SLICES) --
# fused parity tests, then A/B of the C3 / C2 driver-form bench against the fixed snake order.
#   OUT=r06i bash tools/gpu_r06i.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r06i}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $G/pytest_fused.log 2>&1; rc=$?
  tail -3 $G/pytest_fused.log
  faulted $G/pytest_fused.log && stop 99 pytest-fault
  [ $rc -ne 0 ] && stop $rc pytest
fi
for rep in 1 2 3; do
  for lib in default ab/libqsc_nodyn.so; do
    if [ $lib = default ]; then lp=""; else lp="QSC_LIB_PATH=$lib"; fi
    env $lp timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 200 --warmup 20 > $G/ab.log 2>&1 || { tail -5 $G/ab.log; stop 1 ab_c3; }
    tail -1 $G/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('c3 %-22s' % '$lib', round(d['value']), {x: round(v, 2) for x, v in k.items() if x.endswith('_us') and v})" | tee -a $G/ab_dyn.log
  done
done
for lib in default ab/libqsc_nodyn.so; do
  if [ $lib = default ]; then lp=""; else lp="QSC_LIB_PATH=$lib"; fi
  env $lp timeout -k 10 300 python bench.py --config c2 --cpu-baseline 0 --steps 200 --warmup 20 > $G/ab.log 2>&1 || { tail -5 $G/ab.log; stop 1 ab_c2; }
  tail -1 $G/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('c2 %-22s' % '$lib', round(d['value']), {x: round(v, 2) for x, v in k.items() if x.endswith('_us') and v})" | tee -a $G/ab_dyn.log
done
echo SESSION_DONE
