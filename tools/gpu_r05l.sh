#!/bin/bash
# Round-5 session l: early-reads A/B on the other configs, SQ counter passes and HBM-traffic
# passes of the default build, and the quality runs.   OUT=r05l bash tools/gpu_r05l.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-r05l}
G=$R/gpurun_out/$OUT
mkdir -p $G
export TMPDIR=/tmp
stop() { echo "STOP rc=$1 at $2"; exit $1; }
cd $R
echo "# HEAD $(cat .head_sha 2>/dev/null)" > $G/head.txt
for c in c4k c2 c5; do
  REPS=2 BENCH_ARGS="--config $c" timeout -k 10 600 bash tools/gpu_ab.sh variants/libqsc_early4.so > $G/ab_$c.log 2>&1 || { cat $G/ab_$c.log; stop 1 ab_$c; }
  echo "== $c"; cat $G/ab_$c.log
done
OUT=$OUT/pmc_sq timeout -k 10 600 bash tools/pmc_sq2.sh > $G/pmc_sq.log 2>&1 || { cat $G/pmc_sq.log; stop 1 pmc_sq; }
python tools/pmc_summary.py $G/pmc_sq > $G/pmc_sq_summary.txt && grep -A30 scfused $G/pmc_sq_summary.txt | head -32
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "scfused|spass|cpass|cfinish" -d $G/pmc_$c -o run --output-format csv -- python3 $R/tools/prof_passes.py --iters 20 > $G/pmc_$c.log 2>&1 || stop $? pmc_$c
done
cd $R
python tools/traffic.py $G $G/traffic.json
timeout -k 10 600 python -u tools/quality.py > $G/quality.json 2> $G/quality.err || { tail -20 $G/quality.err; stop 1 quality; }
cat $G/quality.err | tail -12
echo SESSION_DONE
