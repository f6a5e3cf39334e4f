#!/bin/bash
# Round-6 session a: rank-16 C-pass on 8-wave workgroups (no VGPR spills) -- the rank-12/16
# parity tests, the c4k K-slab per-GPU sequence and the C4 / C3 driver-form benches.
#   OUT=r06a bash tools/gpu_r06a.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r06a}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kslab.py tests/test_gpu_c4_lockstep.py tests/test_gpu_fused.py -x -v --timeout 300 --timeout-method thread -k "kslab or lockstep or bitexact or c4" > $G/pytest_r16.log 2>&1; rc=$?
tail -3 $G/pytest_r16.log
faulted $G/pytest_r16.log && stop 99 pytest-fault
[ $rc -ne 0 ] && stop $rc pytest
for c in c4k; do
  timeout -k 10 400 python bench.py --config $c --solver kslab --cpu-baseline 0 --steps 200 --warmup 20 > $G/bench_${c}_kslab.log 2>&1 || { tail -5 $G/bench_${c}_kslab.log; stop 1 bench_$c; }
  tail -1 $G/bench_${c}_kslab.log | cut -c1-300
done
for c in c4k c4; do
  timeout -k 10 400 python bench.py --config $c --cpu-baseline 0 --steps 200 --warmup 20 > $G/bench_${c}.log 2>&1 || { tail -5 $G/bench_${c}.log; stop 1 bench_$c; }
  tail -1 $G/bench_${c}.log | cut -c1-300
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $G/bench_c3_driver_form.log 2>&1 || { tail -5 $G/bench_c3_driver_form.log; stop 1 bench_c3; }
tail -1 $G/bench_c3_driver_form.log | cut -c1-300
echo SESSION_DONE
