#!/bin/bash
# Round-5 session c: the C5 bench + its kernel trace, then the 8-rank gloo rehearsal of the C4
# strong K-slab bench (ranks share the card).   OUT=r05c bash tools/gpu_r05c.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r05c}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
cd $R
if [ -x tools/micro/grid_sync ]; then
  timeout -k 5 60 ./tools/micro/grid_sync > $G/grid_sync.log 2>&1 || { cat $G/grid_sync.log; stop 1 grid_sync; }
  cat $G/grid_sync.log
fi
echo "# HEAD $(cat .head_sha 2>/dev/null)" > $G/head.txt
timeout -k 10 400 python bench.py --config c5 --steps 200 --warmup 20 > $G/bench_c5.log 2>&1 || { tail -20 $G/bench_c5.log; stop 1 bench_c5; }
tail -1 $G/bench_c5.log | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/prof_c5 -o run --output-format csv -- python3 $R/bench.py --config c5 --cpu-baseline 0 > $G/bench_c5_prof.log 2>&1 || stop $? rocprof_c5
cd $R
QSC_BENCH_VERBOSE=1 QSC_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 8 --scaling strong --config c4 --shard kslab --steps 4 --warmup 2 --no-extra > $G/rehearse_n8_c4_kslab.log 2>&1 || { tail -30 $G/rehearse_n8_c4_kslab.log; stop 1 rehearse; }
tail -1 $G/rehearse_n8_c4_kslab.log | cut -c1-300
echo SESSION_DONE
