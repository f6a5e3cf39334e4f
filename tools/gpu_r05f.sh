#!/bin/bash
# Round-5 session f: the persistent loop with the split C-finish -- its bit-exactness tests,
# then the C3 bench without / with it (A/B, REPS rounds) and a kernel trace of the loop form,
# then (FULL=1) the whole GPU suite.   OUT=r05f [REPS=2] [FULL=1] bash tools/gpu_r05f.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r05f}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
cd $R
echo "# HEAD $(cat .head_sha 2>/dev/null)" > $G/head.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -k "persistent_loop" -x -v --timeout 120 --timeout-method thread > $G/pytest_loop.log 2>&1 || { tail -30 $G/pytest_loop.log; stop 1 pytest_loop; }
tail -1 $G/pytest_loop.log
for i in $(seq 1 ${REPS:-2}); do
  for e in 0 1; do
    QSC_LOOP=$e timeout -k 10 300 python bench.py --cpu-baseline 0 > $G/bench_c3_loop${e}_$i.log 2>&1 || { tail -20 $G/bench_c3_loop${e}_$i.log; stop 1 bench_loop$e; }
    echo "loop=$e $(tail -1 $G/bench_c3_loop${e}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel"][:14], d["roofline"]["avg_us"], d["roofline"]["frac"], d["kernels"]["scfused_us"], d["kernels"]["cfinish_us"])')"
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/prof_loop -o run --output-format csv -- python3 $R/bench.py --cpu-baseline 0 > $G/bench_prof_loop.log 2>&1 || stop $? rocprof_loop
cd $R
if [ "${FULL:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $G/pytest_gpu.log 2>&1 || { tail -30 $G/pytest_gpu.log; stop 1 pytest; }
  tail -2 $G/pytest_gpu.log
fi
echo SESSION_DONE
