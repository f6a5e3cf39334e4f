#!/bin/bash
# GPU parity of the fused passes + variant timings (tools/tune_variants.py), stopping on faults.
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_fused.py tests/test_gpu_ops.py -q -x > gpurun_out/pt.log 2>&1; rc=$?
tail -3 gpurun_out/pt.log
grep -qE "illegal memory|Memory access fault|HSA_STATUS_ERROR" gpurun_out/pt.log && exit 99
[ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python tools/tune_variants.py run > gpurun_out/tune.log 2>&1; rc=$?
cut -c1-150 gpurun_out/tune.log
exit $rc
