#!/bin/bash
# Round-6 session b: rank-16 tile C-pass variants (waves per workgroup, units per tile) on the
# c4k K-slab share, and the tile size of the c3k8 K-slab share (its C-pass vs C-finish).
#   OUT=r06b bash tools/gpu_r06b.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r06b}
G=$R/gpurun_out/$OUT
mkdir -p $G
cd $R
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_kslab.py tests/test_gpu_c4_lockstep.py tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread > $G/pytest_kslab.log 2>&1; rc=$?
tail -3 $G/pytest_kslab.log
faulted $G/pytest_kslab.log && exit 99
[ $rc -ne 0 ] && exit $rc
summ() { python -c "
import json,sys
d=json.loads(open('$1').read().strip().split('\n')[-1])
k=d['kslab_iteration']
print('$2', round(d['value']), {n: round(v['us'],2) for n,v in k['kernels'].items()})"; }
for v in w8u16 w8u8 w12u12 w16u16; do
  QSC_LIB_PATH=ab/libqsc_$v.so timeout -k 10 300 python bench.py --config c4k --solver kslab --cpu-baseline 0 --steps 200 --warmup 20 > $G/c4k_$v.log 2>&1 || { tail -5 $G/c4k_$v.log; exit 1; }
  summ $G/c4k_$v.log c4k_$v
done
for t in 256 512 1024; do
  QSC_CTILE=$t timeout -k 10 300 python bench.py --config c3k8 --solver kslab --cpu-baseline 0 --steps 200 --warmup 20 > $G/c3k8_t$t.log 2>&1 || { tail -5 $G/c3k8_t$t.log; exit 1; }
  summ $G/c3k8_t$t.log c3k8_t$t
done
echo SESSION_DONE
