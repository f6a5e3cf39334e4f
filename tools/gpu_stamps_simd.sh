#!/bin/bash
# Per-SIMD phase timelines of the fused launch for stamp-instrumented variant libraries:
#   LIBS="variants/libqsc_stamps.so variants/libqsc_nomath.so" bash tools/gpu_stamps_simd.sh
mkdir -p gpurun_out
for lib in ${LIBS:-variants/libqsc_stamps.so}; do
  echo "== $lib"
  QSC_LIB_PATH=$lib timeout -k 10 200 python tools/stamps_simd.py > gpurun_out/stamps_$(basename $lib .so).txt 2>&1 || { tail gpurun_out/stamps_$(basename $lib .so).txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/stamps_$(basename $lib .so).txt | tail -8
done
