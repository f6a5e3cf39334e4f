#!/bin/bash
# One GPU session: tests, smoke, bench, rocprof kernel trace.  Each GPU step has its own limit
# and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -3 gpurun_out/bench.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 --cpu-baseline 0 > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log; exit 1; }
echo PROF_DONE
