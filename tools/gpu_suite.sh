#!/bin/bash
# GPU suite + smoke + single-GPU bench lines of the three configs (no CPU leg):
#   OUT=r02b bash tools/gpu_suite.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
G=$R/gpurun_out/${OUT:-suite}
mkdir -p $G
cd $R
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $G/pytest_gpu.log 2>&1; rc=$?
tail -3 $G/pytest_gpu.log
faulted $G/pytest_gpu.log && { echo FAULT; exit 99; }
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $G/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $G/smoke.log 2>&1 || exit $?
tail -1 $G/smoke.log
for c in c3 c4 c2; do
  timeout -k 10 300 python bench.py --config $c --cpu-baseline 0 > $G/bench_$c.log 2>&1 || exit $?
  tail -1 $G/bench_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$c', round(d['value']), k.get('launches_per_iteration'), {x: round(v, 2) for x, v in k.items() if x.endswith('_us') and v})"
done
