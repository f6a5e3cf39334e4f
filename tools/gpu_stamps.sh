#!/bin/bash
# Phase timelines of the fused launch for stamp-instrumented variant libraries:
#   LIBS="variants/libqsc_stamps.so variants/libqsc_st_nomath.so" bash tools/gpu_stamps.sh
mkdir -p gpurun_out
for lib in ${LIBS:-variants/libqsc_stamps.so}; do
  echo "== $lib"
  QSC_LIB_PATH=$lib timeout -k 10 200 python tools/stamps_f.py 2>&1 | grep -v amdgpu.ids || exit $?
done
