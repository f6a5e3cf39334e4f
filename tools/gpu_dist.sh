#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dist.log 2>&1
rc=$?; tail -3 gpurun_out/dist.log; exit $rc
