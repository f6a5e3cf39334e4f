#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -v -k bitexact --timeout 120 --timeout-method thread > gpurun_out/fz2.log 2>&1
rc=$?; grep -E "PASS|FAIL" gpurun_out/fz2.log | tail -9; exit $rc
