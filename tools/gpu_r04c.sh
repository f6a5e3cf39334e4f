#!/bin/bash
# Round-4 fused-finish / persistent-loop check on small workgroups: the fin and loop parity
# tests, then bench A/B at C2 (default tile and 256-position tiles, where the loop applies) and
# C3.  OUT=gpurun_out/t24 bash tools/gpu_r04c.sh
OUT=${OUT:-gpurun_out/r04c}
mkdir -p $OUT
if [ -x tools/micro/atomic_contention ]; then
  timeout -k 5 60 ./tools/micro/atomic_contention > $OUT/atomic_contention.log 2>&1 || { cat $OUT/atomic_contention.log; exit 1; }
  cat $OUT/atomic_contention.log
fi
echo "# HEAD $(cat .head_sha)" > $OUT/pytest_fin_loop.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 \
  --timeout-method thread -k "fused_finish or persistent_loop" >> $OUT/pytest_fin_loop.log 2>&1 \
  || { tail -20 $OUT/pytest_fin_loop.log; exit 1; }
tail -2 $OUT/pytest_fin_loop.log
REPS=2 ENVS="QSC_FIN=0 QSC_FIN=1" BENCH_ARGS="--config c2" timeout -k 10 300 \
  bash tools/gpu_ab.sh > $OUT/ab_c2.log 2>&1 || { cat $OUT/ab_c2.log; exit 1; }
cat $OUT/ab_c2.log
REPS=2 ENVS="QSC_CTILE=256 QSC_CTILE=256,QSC_FIN=1 QSC_CTILE=256,QSC_LOOP=1" BENCH_ARGS="--config c2" \
  timeout -k 10 400 bash tools/gpu_ab.sh > $OUT/ab_c2_t256.log 2>&1 || { cat $OUT/ab_c2_t256.log; exit 1; }
cat $OUT/ab_c2_t256.log
REPS=2 ENVS="QSC_FIN=0 QSC_FIN=1 QSC_LOOP=1" BENCH_ARGS="--config c3" timeout -k 10 500 \
  bash tools/gpu_ab.sh > $OUT/ab_c3.log 2>&1 || { cat $OUT/ab_c3.log; exit 1; }
cat $OUT/ab_c3.log
