#!/bin/bash
# SPA / NNLS timings + rocprofv3 kernel stats (C3 shape)
mkdir -p gpurun_out/spa_prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/bench_spa.py > gpurun_out/spa_bench.json 2> gpurun_out/spa_bench.err || exit $?
cat gpurun_out/spa_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/spa_prof -o spa -- python tools/bench_spa.py > gpurun_out/spa_prof.log 2>&1 || exit $?
find gpurun_out/spa_prof -name "*kernel_stats.csv" | head -3
