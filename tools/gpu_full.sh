#!/bin/bash
# full GPU suite, then the bench line (stops on the first failure)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full.log 2>&1
rc=$?; tail -3 gpurun_out/full.log
grep -qE "illegal memory|Memory access fault|HSA_STATUS_ERROR" gpurun_out/full.log && exit 99
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/full_bench.log 2>&1 || exit $?
tail -1 gpurun_out/full_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), d['kernels']['scfused_us'], d['kernels']['cfinish_us'])"
done
