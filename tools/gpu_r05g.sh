#!/bin/bash
# Round-5 session g: the whole GPU suite, the fused-launch timeline (stamps build), the C3 bench
# (REPS times) and its kernel trace.   OUT=r05g [REPS=2] [SKIP_TESTS=1] bash tools/gpu_r05g.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r05g}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
cd $R
echo "# HEAD $(cat .head_sha 2>/dev/null)" > $G/head.txt
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $G/pytest_gpu.log 2>&1 || { tail -30 $G/pytest_gpu.log; stop 1 pytest; }
  tail -1 $G/pytest_gpu.log
fi
if [ -f variants/libqsc_stamps.so ]; then
  QSC_LIB_PATH=variants/libqsc_stamps.so timeout -k 10 120 python -u tools/stamps_f.py > $G/stamps_f.log 2>&1 || { tail -20 $G/stamps_f.log; stop 1 stamps; }
  cat $G/stamps_f.log
fi
for i in $(seq 1 ${REPS:-2}); do
  timeout -k 10 300 python bench.py --cpu-baseline 0 > $G/bench_c3_$i.log 2>&1 || { tail -20 $G/bench_c3_$i.log; stop 1 bench; }
  tail -1 $G/bench_c3_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]; print("bench", d["value"], d["ms_per_step"], d["roofline"]["avg_us"], d["roofline"]["frac"], "cfinish", k["cfinish_us"], "spass", k["spass_us"], "cpass", k["cpass_us"])'
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/prof -o run --output-format csv -- python3 $R/bench.py --cpu-baseline 0 > $G/bench_prof.log 2>&1 || stop $? rocprof
cd $R
python - <<'PY' "$G/prof"
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("%-40s calls %6s avg %8.2f us" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
echo SESSION_DONE
