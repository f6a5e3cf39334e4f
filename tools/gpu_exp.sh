#!/bin/bash
# A/B of variant libraries (tools/gpu_ab.sh) followed by stamp timelines of stamp builds:
#   AB="variants/libqsc_a.so ..." ST="variants/libqsc_st_a.so ..." bash tools/gpu_exp.sh
mkdir -p gpurun_out
REPS=${REPS:-2} bash tools/gpu_ab.sh ${AB} || exit $?
for lib in ${ST}; do
  echo "== $lib"
  QSC_LIB_PATH=$lib timeout -k 10 200 python tools/stamps_f.py 2>&1 | grep -v amdgpu.ids || exit $?
  QSC_LIB_PATH=$lib timeout -k 10 200 python tools/stamps_simd.py > gpurun_out/$(basename $lib .so).simd.txt 2>&1 || exit $?
done
