#!/bin/bash
# aux-kernel parity (maps, SPA, NNLS), then timings + rocprofv3 kernel stats of the timing run
mkdir -p gpurun_out/aux_prof
timeout -k 10 240 python -u -m pytest tests/test_gpu_maps.py tests/test_gpu_spa.py tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/aux_tests.log 2>&1
rc=$?; tail -2 gpurun_out/aux_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_spa.py > gpurun_out/aux_bench.json 2> gpurun_out/aux_bench.err || exit $?
cat gpurun_out/aux_bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/aux_prof -o aux --output-format csv -- python tools/bench_spa.py > gpurun_out/aux_prof.log 2>&1
