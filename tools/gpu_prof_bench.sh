#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run (no CPU leg)
mkdir -p gpurun_out/pb
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pb -o run --output-format csv -- python3 bench.py --cpu-baseline 0 ${BENCH_ARGS} > gpurun_out/pb/bench.log 2>&1 || exit $?
tail -1 gpurun_out/pb/bench.log | cut -c1-300
