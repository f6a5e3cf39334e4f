#!/bin/bash
# One GPU session: tests, smoke, bench, rocprof kernel trace.  Each GPU step has its own time
# limit; a crash / abort / timeout (rc >= 124) or any sign of a GPU fault in a log stops the
# chain (plain test failures do not).
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "STOP after rc=$1 in $2"; exit $1; }
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
timeout -k 10 900 python -m pytest tests -m gpu -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -ge 124 ] && stop $rc pytest
faulted gpurun_out/pytest_gpu.log && stop 99 pytest-gpu-fault
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
tail -5 gpurun_out/smoke.log
[ $rc -ne 0 ] && stop $rc smoke
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; rc=$?
tail -3 gpurun_out/bench.log
[ $rc -ne 0 ] && stop $rc bench
if [ -n "$PROFILE" ]; then
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 --cpu-baseline 0 > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log 2>&1 || stop $? rocprof
  echo PROF_DONE
fi
