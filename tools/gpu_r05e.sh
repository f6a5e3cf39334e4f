#!/bin/bash
# Round-5 session e: grid-sync micro (incl. one launch per iteration with head combine), then
# the whole GPU suite at HEAD.   OUT=r05e bash tools/gpu_r05e.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r05e}
G=$R/gpurun_out/$OUT
mkdir -p $G
stop() { echo "STOP rc=$1 at $2"; exit $1; }
cd $R
echo "# HEAD $(cat .head_sha 2>/dev/null)" > $G/head.txt
timeout -k 5 60 ./tools/micro/grid_sync > $G/grid_sync.log 2>&1 || { cat $G/grid_sync.log; stop 1 grid_sync; }
cat $G/grid_sync.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $G/pytest_gpu.log 2>&1 || { tail -30 $G/pytest_gpu.log; stop 1 pytest; }
tail -2 $G/pytest_gpu.log
echo SESSION_DONE
