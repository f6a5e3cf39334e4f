#!/bin/bash
# Round-5 session m: the other BASELINE configs' bench lines at the final HEAD, and the driver's
# default multi-rank commands rehearsed over gloo on one GPU (N = 2 and 4, C3 strong K-slab).
#   OUT=r05am bash tools/gpu_r05m.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r05am}
G=$R/gpurun_out/$OUT
mkdir -p $G
stop() { echo "STOP rc=$1 at $2"; exit $1; }
cd $R
for c in c2 c5 c4k; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --cpu-baseline 0 > $G/bench_$c.log 2>&1 || { tail -20 $G/bench_$c.log; stop 1 bench_$c; }
  tail -1 $G/bench_$c.log | cut -c1-200
done
for n in 2 4; do
  QSC_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus $n --steps 6 --warmup 2 > $G/rehearse_n${n}_c3_kslab.log 2>&1 || { tail -30 $G/rehearse_n${n}_c3_kslab.log; stop 1 rehearse_$n; }
  tail -1 $G/rehearse_n${n}_c3_kslab.log | cut -c1-200
done
echo SESSION_DONE
