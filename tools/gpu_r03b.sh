#!/bin/bash
# Round-3 GPU session B: the GPU suite once with the QSC_DEBUG=1 library (bounds checks read
# back after every call), bench lines at the other configs, and the quality runs.
#   OUT=s7 [SKIP_DEBUG=1] [CFGS="c2 c4k c4" | CFGS=-] [SKIP_QUALITY=1] [QUALITY_ARGS=...]
#   [REHEARSE=1] bash tools/gpu_r03b.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-s7}
G=$R/gpurun_out/$OUT
mkdir -p $G
stop() { echo "STOP rc=$1 at $2"; exit $1; }
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
cd $R
if [ -z "$SKIP_DEBUG" ]; then
  QSC_LIB_PATH=$R/quantized_spectrum_cartography_amd/libqsc_hip_debug.so QSC_DEBUG_CHECK=1 \
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $G/pytest_gpu_debug.log 2>&1; rc=$?
  tail -3 $G/pytest_gpu_debug.log
  faulted $G/pytest_gpu_debug.log && stop 99 debug-fault
  [ $rc -ne 0 ] && { grep -E "^FAILED|Error" $G/pytest_gpu_debug.log | head -20; stop $rc debug; }
fi
for cfg in ${CFGS:-c2 c4k c4}; do
  [ "$cfg" = "-" ] && continue
  timeout -k 10 300 python bench.py --cpu-baseline 0 --config $cfg > $G/bench_$cfg.log 2>&1 || { tail -5 $G/bench_$cfg.log; stop 1 bench-$cfg; }
  tail -1 $G/bench_$cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$cfg', round(d['value']), 'frac', round(d['roofline']['frac'], 4), 'launches', k['launches_per_iteration'], {x: round(v, 2) for x, v in k.items() if x.endswith('_us') and v})"
done
if [ -z "$SKIP_QUALITY" ]; then
  timeout -k 10 600 python tools/quality.py ${QUALITY_ARGS} > $G/quality.json 2> $G/quality.err || { tail -5 $G/quality.err; stop 1 quality; }
  tail -c 1500 $G/quality.json
fi
if [ -n "$REHEARSE" ]; then
  # the driver's plain command with --gpus N > 1 (bench.py spawns its ranks), ranks sharing the
  # one GPU over gloo; both multi-GPU layouts at N = 8
  for run in "2 ijslab" "8 ijslab" "8 kslab"; do
    set -- $run
    QSC_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus $1 --shard $2 --steps 20 --warmup 6 --cpu-baseline 0 > $G/rehearse_n$1_$2.log 2>&1 || { tail -5 $G/rehearse_n$1_$2.log; stop 1 rehearse-$1-$2; }
    faulted $G/rehearse_n$1_$2.log && stop 99 rehearse-fault
    tail -1 $G/rehearse_n$1_$2.log | cut -c1-400
  done
fi
echo SESSION_DONE
