#!/bin/bash
# One GPU session: GPU tests, smoke, bench, rocprofv3 kernel-trace summary of the bench, and the
# HBM-traffic counter passes (FETCH_SIZE, WRITE_SIZE: one --pmc pass each) of the same bench.
# Every GPU step has its own time limit; any crash / abort / timeout / fault ends the chain.
#   OUT=r01 [SKIP_TESTS=1] [NO_PMC=1] bash tools/gpu_round.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r01}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $G/pytest_gpu.log 2>&1; rc=$?
  tail -4 $G/pytest_gpu.log
  faulted $G/pytest_gpu.log && stop 99 pytest-fault
  [ $rc -ne 0 ] && stop $rc pytest
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $G/smoke.log 2>&1 || stop $? smoke
  tail -2 $G/smoke.log
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS} > $G/bench.log 2>&1 || stop $? bench
tail -1 $G/bench.log
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $G/prof -o run --output-format csv -- python3 $R/bench.py --cpu-baseline 0 ${BENCH_ARGS} > $G/bench_prof.log 2>&1 || stop $? rocprof
tail -1 $G/bench_prof.log
if [ -z "$NO_PMC" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "scfused|spass|cpass|cfinish" -d $G/pmc_$c -o run --output-format csv -- python3 $R/tools/prof_passes.py --iters 20 > $G/pmc_$c.log 2>&1 || stop $? pmc_$c
    echo "pmc $c ok"
  done
fi
echo ROUND_DONE
