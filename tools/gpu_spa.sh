#!/bin/bash
# GPU parity of the SPA / SYRK / NNLS kernels, then their C3-shape timings
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_spa.py -x -v --timeout 120 --timeout-method thread > gpurun_out/spa.log 2>&1
rc=$?
tail -4 gpurun_out/spa.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_spa.py
