#!/bin/bash
# Fused-finish bring-up session: the GPU suite with the launch pairs (the default), one small
# fused-finish probe, the suite with it (QSC_FIN=1), then the C3 bench without and with it.  Every GPU step
# has its own time limit; a fault, abort or timeout ends the chain.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-s15}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $G/pytest_pairs.log 2>&1; rc=$?
tail -2 $G/pytest_pairs.log
faulted $G/pytest_pairs.log && stop 99 pairs-fault
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $G/pytest_pairs.log | head -20; stop $rc pairs; }
timeout -k 10 120 python -u tools/probe/fin_probe.py > $G/probe.log 2>&1; rc=$?
cat $G/probe.log | grep -v amdgpu.ids
faulted $G/probe.log && stop 99 probe-fault
[ $rc -ne 0 ] && stop $rc probe
QSC_FIN=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $G/pytest_fin.log 2>&1; rc=$?
tail -2 $G/pytest_fin.log
faulted $G/pytest_fin.log && stop 99 fin-fault
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $G/pytest_fin.log | head -20; stop $rc fin; }
for e in - QSC_FIN=1 - QSC_FIN=1; do
  if [ "$e" = "-" ]; then ev=""; else ev="$e"; fi
  env $ev timeout -k 10 300 python bench.py --cpu-baseline 0 > $G/bench_$e.log 2>&1 || { tail -5 $G/bench_$e.log; stop 1 bench; }
  faulted $G/bench_$e.log && stop 99 bench-fault
  tail -1 $G/bench_$e.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$e', round(d['value']), round(d['ms_per_step']*1e3, 2), 'us/step', {x: round(v, 2) for x, v in k.items() if x.endswith('_us') and v})"
done
if [ -z "$NO_PROF" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/prof -o run --output-format csv -- python3 $R/bench.py --cpu-baseline 0 > $G/bench_prof.log 2>&1 || stop $? rocprof
  cd $R
fi
echo SESSION_DONE
