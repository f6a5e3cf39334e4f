#!/bin/bash
# Round-6 session d: the closing evidence at HEAD -- driver-form C3 bench + its rocprofv3 kernel
# trace, the HBM-traffic counter passes of the fused launch, the multi-rank bench rehearsed over
# gloo on this one card (N = 2, 4: the line carries the K-slab breakdown at world N), and the
# other configs' bench lines.
#   OUT=r06d bash tools/gpu_r06d.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r06d}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
cd $R
echo "# HEAD $(cat .head_sha 2>/dev/null)" > $G/head.txt
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $G/bench_driver_form.log 2>&1 || { tail -20 $G/bench_driver_form.log; stop 1 bench; }
tail -1 $G/bench_driver_form.log | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/prof -o run --output-format csv -- python3 $R/bench.py --cpu-baseline 0 --steps 20 --warmup 5 > $G/bench_prof.log 2>&1 || stop $? rocprof
# the in-sequence figure: 400 timed steps, the roofline's self-replays cut to one launch
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/prof_seq -o run --output-format csv -- python3 $R/bench.py --cpu-baseline 0 --steps 400 --warmup 20 --kernel-reps 1 > $G/bench_prof_seq.log 2>&1 || stop $? rocprof_seq
cd $R
f=$(find $G/prof_seq -name "*kernel_stats.csv" | head -1)
python tools/inseq.py $f $G/inseq.json "$(cat .head_sha 2>/dev/null)"
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "scfused|spass|cpass|cfinish" -d $G/pmc_$c -o run --output-format csv -- python3 $R/tools/prof_passes.py --iters 20 > $G/pmc_$c.log 2>&1 || stop $? pmc_$c
done
cd $R
python tools/traffic.py $G $G/traffic.json | tail -3
for n in 2 4; do
  QSC_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus $n --steps 20 --warmup 4 --cpu-baseline 0 --no-extra > $G/rehearse_n${n}_c3_kslab_gloo.log 2>&1 || { tail -20 $G/rehearse_n${n}_c3_kslab_gloo.log; stop 1 rehearse_$n; }
  tail -1 $G/rehearse_n${n}_c3_kslab_gloo.log | cut -c1-400
done
summ() { python -c "
import json,sys
d=json.loads(open('$1').read().strip().split('\n')[-1])
k=d['kslab_iteration']
print('$2', round(d['value']), {n: round(v['us'],2) for n,v in k['kernels'].items()})"; }
for t in 512 1024 256; do
  QSC_CTILE=$t timeout -k 10 300 python bench.py --config c4k --solver kslab --cpu-baseline 0 --steps 200 --warmup 20 > $G/c4k_kslab_t$t.log 2>&1 || { tail -5 $G/c4k_kslab_t$t.log; stop 1 c4k_t$t; }
  summ $G/c4k_kslab_t$t.log c4k_kslab_t$t
done
for c in c2 c5 c4k c4; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --cpu-baseline 0 > $G/bench_${c}_driver_form.log 2>&1 || { tail -5 $G/bench_${c}_driver_form.log; stop 1 bench_$c; }
  tail -1 $G/bench_${c}_driver_form.log | cut -c1-200
done
for fl in "" "--benchmark"; do
  timeout -k 10 200 python tools/dip_iter.py --iters 100 $fl > $G/dip_iter$fl.log 2>&1 || { tail -5 $G/dip_iter$fl.log; stop 1 dip_iter; }
  tail -1 $G/dip_iter$fl.log
done
timeout -k 10 300 python bench.py --config c5dip --steps 400 --warmup 20 > $G/bench_c5dip.log 2>&1 || { tail -5 $G/bench_c5dip.log; stop 1 bench_c5dip; }
tail -1 $G/bench_c5dip.log | cut -c1-300
echo SESSION_DONE
