#!/bin/bash
# Round-5 baseline session: driver-form bench (no CPU leg), its rocprofv3 kernel-trace summary,
# then the SQ counter groups of the fused launch (one --pmc pass each, tools/pmc_sq2.sh).
#   OUT=r05a bash tools/gpu_r05.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r05a}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
cd $R
echo "# HEAD $(cat .head_sha 2>/dev/null)" > $G/head.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 ${BENCH_ARGS} > $G/bench.log 2>&1 || stop $? bench
tail -1 $G/bench.log | cut -c1-400
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --cpu-baseline 0 ${BENCH_ARGS} > $G/bench_prof.log 2>&1 || stop $? rocprof
cd $R
if [ -z "$NO_PMC" ]; then
  OUT=$OUT/pmc_sq timeout -k 10 900 bash tools/pmc_sq2.sh > $G/pmc.log 2>&1 || { tail -5 $G/pmc.log; stop 1 pmc; }
  tail -1 $G/pmc.log
fi
echo SESSION_DONE
