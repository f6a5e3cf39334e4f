#!/bin/bash
# Round-6 session p: rocprofv3 kernel traces of the driver-form bench at HEAD (the committed
# in-sequence figure the bench line reads: profiles/r06/inseq.json).
#   OUT=r06p bash tools/gpu_r06p.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r06p}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/prof -o run --output-format csv -- python3 $R/bench.py --cpu-baseline 0 --steps 20 --warmup 5 > $G/bench_prof.log 2>&1 || stop $? rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $G/prof_seq -o run --output-format csv -- python3 $R/bench.py --cpu-baseline 0 --steps 400 --warmup 20 --kernel-reps 1 > $G/bench_prof_seq.log 2>&1 || stop $? rocprof_seq
cd $R
f=$(find $G/prof_seq -name "*kernel_stats.csv" | head -1)
python tools/inseq.py $f $G/inseq.json "$(cat .head_sha 2>/dev/null)"
cat $G/inseq.json | head -12
echo SESSION_DONE
