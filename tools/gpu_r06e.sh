#!/bin/bash
# Round-6 session e: the DIP iteration with the decoder's Adam as one flat launch
# (qsc_adam_flat) -- its parity tests, the c5dip bench line and a rocprofv3 split.
#   OUT=r06e bash tools/gpu_r06e.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r06e}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_abi.py -v --timeout 300 --timeout-method thread -k "dip or generator or restart or gan or abi or holdout or c5" > $G/pytest_dip.log 2>&1; rc=$?
tail -3 $G/pytest_dip.log
faulted $G/pytest_dip.log && stop 99 pytest-fault
[ $rc -ge 124 ] && stop $rc pytest-timeout
grep -E "^(FAILED|ERROR)" $G/pytest_dip.log | head
for m in weights z; do
  timeout -k 10 200 python -u tools/dip_iter.py --iters 100 --optimize $m > $G/dip_iter_$m.log 2>&1 || { tail -5 $G/dip_iter_$m.log; stop 1 dip_iter_$m; }
  tail -1 $G/dip_iter_$m.log
done
timeout -k 10 200 python -u tools/dip_iter.py --iters 30 --eager > $G/dip_iter_eager.log 2>&1 || { tail -5 $G/dip_iter_eager.log; stop 1 dip_eager; }
tail -1 $G/dip_iter_eager.log
timeout -k 10 300 python bench.py --config c5dip --steps 400 --warmup 20 > $G/bench_c5dip.log 2>&1 || { tail -5 $G/bench_c5dip.log; stop 1 bench_c5dip; }
tail -1 $G/bench_c5dip.log | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/prof_dip -o run --output-format csv -- python3 $R/tools/dip_iter.py --iters 200 > $G/dip_prof.log 2>&1 || stop $? rocprof_dip
cd $R
f=$(find $G/prof_dip -name "*kernel_stats.csv" | head -1)
python tools/kernel_split.py $f 202 $G/dip_split.json | head -4
echo SESSION_DONE
