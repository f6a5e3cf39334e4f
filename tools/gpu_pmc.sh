#!/bin/bash
# Counter passes over tools/prof_passes.py (one rocprofv3 --pmc pass per group, nothing else
# traced).  Usage: OUT=name [QSC_LIB_PATH=variants/libqsc_x.so] bash tools/gpu_pmc.sh "C1 C2 ..." "C3 ..." ...
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=${OUT:-pmc}
mkdir -p $R/gpurun_out/$OUT
cd /tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "scfused|spass|cpass|cfinish" -d $R/gpurun_out/$OUT/g$i -o run --output-format csv -- python3 $R/tools/prof_passes.py --iters 10 > $R/gpurun_out/$OUT/g$i.log 2>&1 || { echo "FAIL group $i rc=$?"; tail -20 $R/gpurun_out/$OUT/g$i.log; exit 1; }
done
echo "ok $OUT"
