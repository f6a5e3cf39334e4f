#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_maps.py tests/test_gpu_spa.py -x -v --timeout 120 --timeout-method thread > gpurun_out/maps.log 2>&1
rc=$?
tail -25 gpurun_out/maps.log
exit $rc
