#!/bin/bash
# Round-6 session h: tile C-pass start / end latencies (persistent rank-16 workgroups with the next
# tile's unit bounds, C column and S rows read during the walk; part-sum bins read ahead; ||C||^2
# from reads under the staging barrier) -- full GPU suite, stamps, A/B against the previous build.
#   OUT=r06h bash tools/gpu_r06h.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r06h}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $G/pytest_gpu.log 2>&1; rc=$?
  tail -3 $G/pytest_gpu.log
  faulted $G/pytest_gpu.log && stop 99 pytest-fault
  [ $rc -ne 0 ] && stop $rc pytest
fi
QSC_LIB_PATH=ab/libqsc_stamps16p.so timeout -k 10 200 python tools/stamps_r16.py > $G/stamps16p.log 2>&1 || { tail -5 $G/stamps16p.log; stop 1 stamps; }
grep -v "from launch\|block starts" $G/stamps16p.log
for rep in 1 2; do
  for c in c4k c3k8; do
    for lib in default ab/libqsc_nopersist.so; do
      if [ $lib = default ]; then lp=""; else lp="QSC_LIB_PATH=$lib"; fi
      env $lp timeout -k 10 300 python bench.py --config $c --solver kslab --cpu-baseline 0 --steps 200 --warmup 20 > $G/ab.log 2>&1 || { tail -5 $G/ab.log; stop 1 ab; }
      tail -1 $G/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kslab_iteration']['kernels']; print('%-5s %-26s' % ('$c', '$lib'), round(d['value']), {x: round(v['us'], 2) for x, v in k.items()})" | tee -a $G/ab_tile.log
    done
  done
done
for lib in default ab/libqsc_nopersist.so; do
  if [ $lib = default ]; then lp=""; else lp="QSC_LIB_PATH=$lib"; fi
  env $lp timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 200 --warmup 20 > $G/ab.log 2>&1 || { tail -5 $G/ab.log; stop 1 ab_c3; }
  tail -1 $G/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('c3    %-26s' % '$lib', round(d['value']), {x: round(v, 2) for x, v in k.items() if x.endswith('_us') and v})" | tee -a $G/ab_tile.log
done
echo SESSION_DONE
