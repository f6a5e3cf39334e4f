#!/bin/bash
# Round-6 session c: the whole GPU suite + smoke, then the bench lines this round changed:
# c5dip (the DIP path as hipGraph chunks), the K-slab shares (reduce-scatter-borne ||C||^2,
# one-round tiles), C3 driver form with the in-sequence fused-launch time.
#   OUT=r06c bash tools/gpu_r06c.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r06c}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $G/pytest_gpu.log 2>&1; rc=$?
  tail -4 $G/pytest_gpu.log
  faulted $G/pytest_gpu.log && stop 99 pytest-fault
  [ $rc -ge 124 ] && stop $rc pytest-timeout
  grep -E "^(FAILED|ERROR)" $G/pytest_gpu.log | head -10
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $G/smoke.log 2>&1 || stop $? smoke
  tail -2 $G/smoke.log
fi
j() { python -c "
import json,sys
d=json.loads(open('$1').read().strip().split('\n')[-1])
rf=d['roofline']
print('$2', round(d['value']), 'frac', round(rf['frac'],3), 'avg_us', round(rf['avg_us'],2), 'self', rf.get('avg_us_self_replay'), 'inseq', rf.get('avg_us_in_sequence'))
for k in ('kslab_iteration','dip_iteration'):
    if d.get(k): print('  ', k, json.dumps(d[k])[:900])
if d['kernels'].get('in_sequence'): print('   in_sequence', d['kernels']['in_sequence'])
"; }
timeout -k 10 400 python bench.py --config c5dip --steps 400 --warmup 20 > $G/bench_c5dip.log 2>&1 || { tail -20 $G/bench_c5dip.log; stop 1 bench_c5dip; }
j $G/bench_c5dip.log c5dip
for c in c3k8 c3k4 c3k2 c4k; do
  timeout -k 10 300 python bench.py --config $c --solver kslab --cpu-baseline 0 --steps 200 --warmup 20 > $G/bench_${c}_kslab.log 2>&1 || { tail -5 $G/bench_${c}_kslab.log; stop 1 bench_$c; }
  j $G/bench_${c}_kslab.log ${c}_kslab
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $G/bench_c3_driver_form.log 2>&1 || { tail -5 $G/bench_c3_driver_form.log; stop 1 bench_c3; }
j $G/bench_c3_driver_form.log c3
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/prof_dip -o run --output-format csv -- python3 $R/tools/dip_iter.py --iters 200 > $G/dip_prof.log 2>&1 || stop $? rocprof_dip
cd $R
tail -1 $G/dip_prof.log
f=$(find $G/prof_dip -name "*kernel_stats.csv" | head -1)
python tools/kernel_split.py $f 202 $G/dip_split.json | head -8
timeout -k 10 200 python tools/dip_iter.py --iters 50 --eager > $G/dip_eager.log 2>&1 || stop $? dip_eager
tail -1 $G/dip_eager.log
echo SESSION_DONE
