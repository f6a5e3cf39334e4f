#!/bin/bash
# Round-6 session f: price the fused launch's LDS bank conflicts at C3 -- diagnostic builds whose
# gathers are made conflict-free (wrong values: timing only; QSC_DIAG_NOCONF_S / _C, which also
# turn off the row-address unpack, so the baseline is the index-form build "noaddr").
#   OUT=r06f bash tools/gpu_r06f.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r06f}
G=$R/gpurun_out/$OUT
mkdir -p $G
cd $R
for rep in 1 2; do
  for v in dev8 noaddr noconfS noconfC noconfSC; do
    QSC_LIB_PATH=ab/libqsc_$v.so timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 400 --warmup 20 > $G/b_$v.log 2>&1 || { tail -5 $G/b_$v.log; exit 1; }
    python -c "
import json
d=json.loads(open('$G/b_$v.log').read().strip().split('\n')[-1])
k=d['kernels']
print('$rep', '$v', round(d['value']), 'scfused', round(k['scfused_us'],2), 'spass', round(k['spass_us'],2), 'cpass', round(k['cpass_us'],2))" | tee -a $G/ab.log
  done
done
echo SESSION_DONE
