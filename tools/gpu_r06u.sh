#!/bin/bash
# Round-6 session u: fused launch with the C units' list metadata staged in LDS -- the fused /
# full-size parity tests, then C3 / C2 / C4 driver-form A/B against the previous build.
#   OUT=r06u bash tools/gpu_r06u.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r06u}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_gpu_capture.py -x -q --timeout 300 --timeout-method thread > $G/pytest.log 2>&1; rc=$?
tail -2 $G/pytest.log
faulted $G/pytest.log && stop 99 pytest-fault
[ $rc -ne 0 ] && stop $rc pytest
for rep in 1 2 3; do
  for lib in default ab/libqsc_headref.so; do
    if [ $lib = default ]; then lp=""; else lp="QSC_LIB_PATH=$lib"; fi
    env $lp timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 200 --warmup 20 > $G/ab.log 2>&1 || { tail -5 $G/ab.log; stop 1 ab_c3; }
    tail -1 $G/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('c3 %-22s' % '$lib', round(d['value']), {x: round(v, 2) for x, v in k.items() if x.endswith('_us') and v})" | tee -a $G/ab_mlds.log
  done
done
for c in c2 c4; do
  for lib in default ab/libqsc_headref.so; do
    if [ $lib = default ]; then lp=""; else lp="QSC_LIB_PATH=$lib"; fi
    env $lp timeout -k 10 300 python bench.py --config $c --cpu-baseline 0 --steps 100 --warmup 10 > $G/ab.log 2>&1 || { tail -5 $G/ab.log; stop 1 ab_$c; }
    tail -1 $G/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$c %-22s' % '$lib', round(d['value']), {x: round(v, 2) for x, v in k.items() if x.endswith('_us') and v})" | tee -a $G/ab_mlds.log
  done
done
echo SESSION_DONE
