#!/bin/bash
# Parity of variant libraries (fused-launch tests + C3 full-size) then an alternating A/B bench
# against the default build:  bash tools/gpu_variant_ab.sh variants/libqsc_a.so ...
mkdir -p gpurun_out/vab
for lib in "$@"; do
  n=$(basename $lib .so)
  QSC_LIB_PATH=$lib timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_fused.py tests/test_gpu_fullsize.py -m gpu -k "bitexact or signed or onebit_config or fused_pass or solver_vs" \
    > gpurun_out/vab/pt_$n.log 2>&1; rc=$?
  tail -2 gpurun_out/vab/pt_$n.log
  grep -qE "illegal memory|Memory access fault|HSA_STATUS_ERROR" gpurun_out/vab/pt_$n.log && exit 99
  [ $rc -ne 0 ] && exit $rc
done
REPS=${REPS:-3} bash tools/gpu_ab.sh "$@"
