#!/bin/bash
# Round-6 session g: persistent rank-16 tile C-pass (next tile's S rows in registers) -- the
# rank-16 parity tests, then the c4k K-slab sequence A/B against the two-round form.
#   OUT=r06g bash tools/gpu_r06g.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r06g}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
cd $R
QSC_LIB_PATH=ab/libqsc_stamps16.so timeout -k 10 200 python tools/stamps_r16.py > $G/stamps16.log 2>&1 || { tail -5 $G/stamps16.log; stop 1 stamps; }
cat $G/stamps16.log
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_kslab.py tests/test_gpu_c4_lockstep.py tests/test_gpu_fused.py -x -v --timeout 300 --timeout-method thread -k "kslab or lockstep or bitexact or c4 or rank" > $G/pytest_r16.log 2>&1; rc=$?
[ -n "$SKIP_TESTS" ] || { tail -3 $G/pytest_r16.log
faulted $G/pytest_r16.log && stop 99 pytest-fault
[ $rc -ne 0 ] && stop $rc pytest; }
for rep in 1 2; do
  for lib in default ab/libqsc_nopersist.so; do
    if [ $lib = default ]; then lp=""; else lp="QSC_LIB_PATH=$lib"; fi
    env $lp timeout -k 10 300 python bench.py --config c4k --solver kslab --cpu-baseline 0 --steps 200 --warmup 20 > $G/ab.log 2>&1 || { tail -5 $G/ab.log; stop 1 ab; }
    tail -1 $G/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kslab_iteration']['kernels']; print('%-32s' % '$lib', round(d['value']), {x: round(v['us'], 2) for x, v in k.items()})" | tee -a $G/ab_persist.log
  done
done
echo SESSION_DONE
