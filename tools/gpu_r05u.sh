#!/bin/bash
# Round-5 session u: the round's evidence at HEAD -- the driver-form C3 bench, its kernel trace,
# SQ counter and HBM-traffic passes, the fused launch's timelines (stamps build).
#   OUT=r05u bash tools/gpu_r05u.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r05u}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
cd $R
echo "# HEAD $(cat .head_sha 2>/dev/null)" > $G/head.txt
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $G/bench_driver_form.log 2>&1 || { tail -20 $G/bench_driver_form.log; stop 1 bench; }
tail -1 $G/bench_driver_form.log | cut -c1-400
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/prof -o run --output-format csv -- python3 $R/bench.py --cpu-baseline 0 > $G/bench_prof.log 2>&1 || stop $? rocprof
cd $R
OUT=$OUT/pmc_sq timeout -k 10 600 bash tools/pmc_sq2.sh > $G/pmc_sq.log 2>&1 || { cat $G/pmc_sq.log; stop 1 pmc_sq; }
python tools/pmc_summary.py $G/pmc_sq > $G/pmc_sq_summary.txt
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "scfused|spass|cpass|cfinish" -d $G/pmc_$c -o run --output-format csv -- python3 $R/tools/prof_passes.py --iters 20 > $G/pmc_$c.log 2>&1 || stop $? pmc_$c
done
cd $R
python tools/traffic.py $G $G/traffic.json
QSC_LIB_PATH=variants/libqsc_stamps.so timeout -k 10 120 python -u tools/stamps_simd.py > $G/stamps_simd.log 2>&1 || { tail -20 $G/stamps_simd.log; stop 1 stamps_simd; }
QSC_LIB_PATH=variants/libqsc_stamps.so timeout -k 10 120 python -u tools/stamps_f.py > $G/stamps_f.log 2>&1 || { tail -20 $G/stamps_f.log; stop 1 stamps_f; }
tail -3 $G/stamps_simd.log
echo SESSION_DONE
