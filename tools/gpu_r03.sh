#!/bin/bash
# One round-3 GPU session: GPU tests + smoke, the C3 bench under each environment setting in
# $ENVS (alternating, A/B), a rocprofv3 kernel-trace summary of the default bench, and the
# LDS / VALU SQ counters of the passes with and without the list schedule.  Every GPU step has
# its own time limit; a fault, abort or timeout ends the chain.
#   OUT=s3 [SKIP_TESTS=1] [NO_PROF=1] [NO_PMC=1] [ENVS="- QSC_SCHEDULE=0"] [REPS=2] bash tools/gpu_r03.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-s3}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > $G/pytest_gpu.log 2>&1; rc=$?
  tail -3 $G/pytest_gpu.log
  faulted $G/pytest_gpu.log && stop 99 pytest-fault
  [ $rc -ne 0 ] && { grep -E "^FAILED|Error" $G/pytest_gpu.log | head -20; stop $rc pytest; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $G/smoke.log 2>&1 || stop $? smoke
  tail -1 $G/smoke.log
fi
i=0
for rep in $(seq ${REPS:-1}); do
  for e in ${ENVS:--}; do
    i=$((i+1))
    if [ "$e" = "-" ]; then ev=""; else ev="${e//,/ }"; fi
    env $ev timeout -k 10 300 python bench.py --cpu-baseline 0 ${BENCH_ARGS} > $G/bench_$i.log 2>&1 || { tail -5 $G/bench_$i.log; stop 1 bench; }
    faulted $G/bench_$i.log && stop 99 bench-fault
    tail -1 $G/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$e', round(d['value']), round(d['roofline']['frac'], 4), {x: round(v, 2) for x, v in k.items() if x.endswith('_us') and v})"
  done
done
if [ -z "$NO_PROF" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/prof -o run --output-format csv -- python3 $R/bench.py --cpu-baseline 0 ${BENCH_ARGS} > $G/bench_prof.log 2>&1 || stop $? rocprof
  tail -1 $G/bench_prof.log | cut -c1-300
  cd $R
fi
if [ -z "$NO_PMC" ]; then
  cd /tmp
  GL="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
  for sch in 1 0; do
    QSC_SCHEDULE=$sch timeout -s KILL 240 rocprofv3 --pmc $GL --kernel-include-regex "scfused|spass|cpass|cfinish" -d $G/pmc_sched$sch -o run --output-format csv -- python3 $R/tools/prof_passes.py --iters 10 > $G/pmc_sched$sch.log 2>&1 || stop $? pmc$sch
    echo "pmc sched=$sch ok"
  done
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "scfused|spass|cpass|cfinish" -d $G/pmc_$c -o run --output-format csv -- python3 $R/tools/prof_passes.py --iters 10 > $G/pmc_$c.log 2>&1 || stop $? pmc_$c
    echo "pmc $c ok"
  done
  cd $R
fi
echo SESSION_DONE
