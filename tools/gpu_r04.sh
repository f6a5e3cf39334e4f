#!/bin/bash
# Round-4 GPU session: HEAD-stamped GPU suite + smoke, a small fused-finish probe first, then the
# C3 bench with the launch pairs and with the fused finish, and a rocprofv3 kernel-trace summary
# of each.  Every GPU step has its own time limit; a fault, abort or timeout ends the chain.
#   OUT=t1 [SKIP_TESTS=1] [NO_PROF=1] [ENVS="QSC_FIN=0 QSC_FIN=1"] [REPS=1] [BENCH_ARGS=...]
#   bash tools/gpu_r04.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-t1}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
HEAD=$(cat $R/.head_sha 2>/dev/null || echo unknown)
stop() { echo "STOP rc=$1 at $2"; exit $1; }
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
cd $R
if [ -z "$SKIP_PROBE" ]; then
  echo "# HEAD $HEAD" > $G/probe.log
  timeout -k 10 120 python -u tools/probe/fin_probe.py >> $G/probe.log 2>&1; rc=$?
  grep -v amdgpu.ids $G/probe.log
  faulted $G/probe.log && stop 99 probe-fault
  [ $rc -ne 0 ] && stop $rc probe
fi
if [ -z "$SKIP_TESTS" ]; then
  echo "# HEAD $HEAD" > $G/pytest_gpu.log
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread ${PYTEST_ARGS} >> $G/pytest_gpu.log 2>&1; rc=$?
  tail -3 $G/pytest_gpu.log
  faulted $G/pytest_gpu.log && stop 99 pytest-fault
  [ $rc -ne 0 ] && { grep -E "^FAILED|Error" $G/pytest_gpu.log | head -20; stop $rc pytest; }
  echo "# HEAD $HEAD" > $G/smoke.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >> $G/smoke.log 2>&1 || stop $? smoke
  tail -1 $G/smoke.log
fi
i=0
for rep in $(seq ${REPS:-1}); do
  for e in ${ENVS:-QSC_FIN=0 QSC_FIN=1}; do
    i=$((i+1))
    if [ "$e" = "-" ]; then ev=""; else ev="${e//,/ }"; fi
    echo "# HEAD $HEAD env $e" > $G/bench_$i.log
    env $ev timeout -k 10 300 python bench.py --cpu-baseline 0 ${BENCH_ARGS} >> $G/bench_$i.log 2>&1 || { tail -5 $G/bench_$i.log; stop 1 bench; }
    faulted $G/bench_$i.log && stop 99 bench-fault
    tail -1 $G/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$e', round(d['value']), round(d['ms_per_step']*1e3, 2), 'us/step', round(d['roofline']['frac'], 4), 'launches', k.get('launches_per_iteration'), {x: round(v, 2) for x, v in k.items() if x.endswith('_us') and v})"
  done
done
if [ -z "$NO_PROF" ]; then
  cd /tmp
  for e in ${PROF_ENVS:-QSC_FIN=0 QSC_FIN=1}; do
    tag=${e//=/}
    env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/prof_$tag -o run --output-format csv -- python3 $R/bench.py --cpu-baseline 0 ${BENCH_ARGS} > $G/bench_prof_$tag.log 2>&1 || stop $? rocprof
    tail -1 $G/bench_prof_$tag.log | cut -c1-200
  done
  cd $R
fi
echo SESSION_DONE
