#!/bin/bash
# Round-6 session x: the bench's timed region led by untimed solver iterations (LEAD_ITERS)
# instead of a device spin -- five driver-form C3 runs, C2, c5dip, c4k K-slab, a gloo N = 2
# rehearsal.
#   OUT=r06x bash tools/gpu_r06x.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r06x}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
cd $R
summ() { python -c "
import json,sys
d=json.loads(open('$1').read().strip().split('\n')[-1])
t=d['timing']
print('$2', round(d['value']), round(d['ms_per_step']*1e3,2), 'us/step; lead', round(t['lead_s']*1e6,1), 'us; host_wall_value', round(t['host_wall_value']))" | tee -a $G/summary.log; }
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $G/c3_$i.log 2>&1 || { tail -5 $G/c3_$i.log; stop 1 c3_$i; }
  summ $G/c3_$i.log c3_run$i
done
timeout -k 10 300 python bench.py --steps 400 --warmup 40 --cpu-baseline 0 > $G/c3_400.log 2>&1 || { tail -5 $G/c3_400.log; stop 1 c3_400; }
summ $G/c3_400.log c3_400steps
for c in c2 c5dip; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --cpu-baseline 0 > $G/$c.log 2>&1 || { tail -5 $G/$c.log; stop 1 $c; }
  summ $G/$c.log $c
done
timeout -k 10 300 python bench.py --config c4k --solver kslab --steps 20 --warmup 5 --cpu-baseline 0 > $G/c4k_kslab.log 2>&1 || { tail -5 $G/c4k_kslab.log; stop 1 c4k; }
summ $G/c4k_kslab.log c4k_kslab
QSC_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 4 --cpu-baseline 0 --no-extra > $G/rehearse_n2.log 2>&1 || { tail -20 $G/rehearse_n2.log; stop 1 rehearse; }
summ $G/rehearse_n2.log gloo_n2
echo SESSION_DONE
