#!/bin/bash
# Round-6 session l: rank-16 tile C-pass without the software-pipelined row gather (124 VGPRs:
# 12 or 16 waves per workgroup fit without spills) -- c4k K-slab sequence A/B.
#   OUT=r06l bash tools/gpu_r06l.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r06l}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
cd $R
for rep in 1 2; do
  for lib in default ab/libqsc_w16np.so ab/libqsc_w12np.so ab/libqsc_w8np.so; do
    if [ $lib = default ]; then lp=""; else lp="QSC_LIB_PATH=$lib"; fi
    env $lp timeout -k 10 300 python bench.py --config c4k --solver kslab --cpu-baseline 0 --steps 200 --warmup 20 > $G/ab.log 2>&1 || { tail -5 $G/ab.log; stop 1 ab; }
    tail -1 $G/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kslab_iteration']['kernels']; print('%-22s' % '$lib', round(d['value']), {x: round(v['us'], 2) for x, v in k.items()})" | tee -a $G/ab_r16_nopf.log
  done
done
echo SESSION_DONE
