#!/bin/bash
# Iteration loop on the GPU box: parity of the hot path (fused passes, full-size configs, ops),
# then a short bench (no CPU baseline) and a rocprofv3 kernel-trace summary of it.
#   OUT=r02x [TESTS="tests/test_gpu_fused.py ..."] [BENCH_ARGS=...] [NO_PROF=1] bash tools/gpu_iter.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-iter}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
cd $R
TESTS=${TESTS:-"tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_gpu_ops.py"}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $G/pytest.log 2>&1; rc=$?
  tail -3 $G/pytest.log
  faulted $G/pytest.log && stop 99 pytest-fault
  [ $rc -ne 0 ] && stop $rc pytest
fi
timeout -k 10 300 python bench.py --cpu-baseline 0 ${BENCH_ARGS} > $G/bench.log 2>&1 || stop $? bench
python -c "import json;d=json.loads(open('$G/bench.log').read().strip().splitlines()[-1]);print('value',round(d['value']),'scfused_us',d['kernels']['scfused_us'],'spass_us',d['kernels']['spass_us'],'cpass_us',d['kernels']['cpass_us'],'cfinish_us',d['kernels']['cfinish_us'],'frac',d['roofline']['frac'],'slf',d['quality']['slf_nmse'])"
if [ -z "$NO_PROF" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/prof -o run --output-format csv -- python3 $R/bench.py --cpu-baseline 0 ${BENCH_ARGS} > $G/bench_prof.log 2>&1 || stop $? rocprof
  echo prof ok
fi
echo ITER_DONE
