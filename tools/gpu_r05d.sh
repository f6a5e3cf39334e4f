#!/bin/bash
# Round-5 session d: DIP oracle test, the K-slab solver's own per-GPU sequence at world 1 over
# RCCL (bench --solver kslab --config c4k: one GPU's share of C4 at N = 8) + its kernel trace.
#   OUT=r05d bash tools/gpu_r05d.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r05d}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
cd $R
echo "# HEAD $(cat .head_sha 2>/dev/null)" > $G/head.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_fused.py -k "dip" > $G/pytest_dip.log 2>&1 || { tail -30 $G/pytest_dip.log; stop 1 pytest; }
tail -2 $G/pytest_dip.log
timeout -k 10 300 python bench.py --config c4k --solver kslab --cpu-baseline 0 > $G/bench_c4k_kslab.log 2>&1 || { tail -20 $G/bench_c4k_kslab.log; stop 1 bench_kslab; }
tail -1 $G/bench_c4k_kslab.log | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/prof_c4k_kslab -o run --output-format csv -- python3 $R/bench.py --config c4k --solver kslab --cpu-baseline 0 > $G/bench_c4k_kslab_prof.log 2>&1 || stop $? rocprof_kslab
echo SESSION_DONE
