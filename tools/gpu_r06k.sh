#!/bin/bash
# Round-6 session k: closing validation at HEAD -- the whole GPU suite, smoke(), the driver-form
# C3 bench (CPU baseline included) and the c5dip line.
#   OUT=r06k bash tools/gpu_r06k.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r06k}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
cd $R
echo "# HEAD $(cat .head_sha 2>/dev/null)" > $G/head.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $G/pytest_gpu.log 2>&1; rc=$?
tail -3 $G/pytest_gpu.log
faulted $G/pytest_gpu.log && stop 99 pytest-fault
[ $rc -ne 0 ] && stop $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $G/smoke.log 2>&1 || { tail -5 $G/smoke.log; stop 1 smoke; }
tail -1 $G/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $G/bench_driver_form.log 2>&1 || { tail -20 $G/bench_driver_form.log; stop 1 bench; }
tail -1 $G/bench_driver_form.log | cut -c1-300
timeout -k 10 400 python bench.py --config c5dip --steps 200 --warmup 20 --cpu-baseline 0 > $G/bench_c5dip.log 2>&1 || { tail -20 $G/bench_c5dip.log; stop 1 bench_c5dip; }
tail -1 $G/bench_c5dip.log | cut -c1-300
echo SESSION_DONE
