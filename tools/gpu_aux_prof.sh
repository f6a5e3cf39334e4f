#!/bin/bash
# SPA / NNLS / map-compose timings (C3 shape) + rocprofv3 kernel stats of the same command
mkdir -p gpurun_out/aux_prof
timeout -k 10 300 python tools/bench_spa.py > gpurun_out/aux_bench.json 2> gpurun_out/aux_bench.err || exit $?
cat gpurun_out/aux_bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/aux_prof -o aux --output-format csv -- python tools/bench_spa.py > gpurun_out/aux_prof.log 2>&1 || exit $?
find gpurun_out/aux_prof -name "*stats*"
