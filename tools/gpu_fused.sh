#!/bin/bash
# fused S-step + C-pass: parity (bit-exact vs the two-launch form), the solver suite, then bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_distributed.py -x -v --timeout 120 --timeout-method thread > gpurun_out/fz.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error" gpurun_out/fz.log | tail -12
grep -qE "illegal memory|Memory access fault|HSA_STATUS_ERROR" gpurun_out/fz.log && exit 99
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/fz_bench.log 2>&1 || exit $?
tail -1 gpurun_out/fz_bench.log | cut -c1-400
