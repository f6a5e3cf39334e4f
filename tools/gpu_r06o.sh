#!/bin/bash
# Round-6 session o: the multi-rank bench at HEAD rehearsed over gloo on this one card (N = 2, 8:
# the driver's SCALE command form, ranks sharing the GPU).
#   OUT=r06o bash tools/gpu_r06o.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r06o}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
cd $R
for n in 2 8; do
  QSC_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus $n --steps 20 --warmup 4 --cpu-baseline 0 --no-extra > $G/rehearse_n${n}_c3_kslab_gloo.log 2>&1 || { tail -20 $G/rehearse_n${n}_c3_kslab_gloo.log; stop 1 rehearse_$n; }
  tail -1 $G/rehearse_n${n}_c3_kslab_gloo.log | python -c "
import json,sys
d=json.loads(sys.stdin.read())
k=d['kslab_iteration']
print($n, round(d['value'],1), d['roofline']['kernel'][:30], {x: round(v['us'],1) for x,v in k['kernels'].items()}, {x: round(v['us'],1) for x,v in k['collectives'].items()}, k.get('projected'))"
done
echo SESSION_DONE
