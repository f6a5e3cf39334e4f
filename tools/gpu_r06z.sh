#!/bin/bash
# Round-6 session z: tile C-pass bin map staged in LDS (part sums), ||C||^2 from the staged C^T
# -- the tile C-pass parity tests, then A/B of the c4k / c3k8 K-slab sequences and C3.
#   OUT=r06z bash tools/gpu_r06z.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r06z}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kslab.py tests/test_gpu_c4_lockstep.py tests/test_gpu_fused.py tests/test_gpu_capture.py tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread > $G/pytest.log 2>&1; rc=$?
tail -2 $G/pytest.log
faulted $G/pytest.log && stop 99 pytest-fault
[ $rc -ne 0 ] && stop $rc pytest
for rep in 1 2; do
  for c in c4k c3k8; do
    for lib in default ab/libqsc_headref.so; do
      if [ $lib = default ]; then lp=""; else lp="QSC_LIB_PATH=$lib"; fi
      env $lp timeout -k 10 300 python bench.py --config $c --solver kslab --cpu-baseline 0 --steps 200 --warmup 20 > $G/ab.log 2>&1 || { tail -5 $G/ab.log; stop 1 ab; }
      tail -1 $G/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kslab_iteration']['kernels']; print('%-5s %-22s' % ('$c', '$lib'), round(d['value']), {x: round(v['us'], 2) for x, v in k.items()})" | tee -a $G/ab_mk.log
    done
  done
done
for lib in default ab/libqsc_headref.so; do
  if [ $lib = default ]; then lp=""; else lp="QSC_LIB_PATH=$lib"; fi
  env $lp timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 200 --warmup 20 > $G/ab.log 2>&1 || { tail -5 $G/ab.log; stop 1 ab_c3; }
  tail -1 $G/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('c3    %-22s' % '$lib', round(d['value']), {x: round(v, 2) for x, v in k.items() if x.endswith('_us') and v})" | tee -a $G/ab_mk.log
done
echo SESSION_DONE
