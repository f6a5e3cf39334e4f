#!/bin/bash
# Round-4 session B: C2 tile sweep (QSC_CTILE x QSC_FIN), the C4 K-slab rehearsal over gloo on one
# GPU (8 ranks share the card), and the C5 exploration runs.  Steps have their own limits; a
# fault or timeout ends the chain.
R=${GRAFT_REPO_ROOT:-$(pwd)}
G=$R/gpurun_out/${OUT:-t4}
mkdir -p $G/rehearsal
cd $R
HEAD=$(cat .head_sha 2>/dev/null || echo unknown)
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
summ() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$2', round(d['value']), round(d['ms_per_step']*1e3, 2), 'us/step', round(d['roofline']['frac'], 4), 'launches', k.get('launches_per_iteration'), {x: round(v, 2) for x, v in k.items() if x.endswith('_us') and v})"; }
if [ -z "$SKIP_C2" ]; then
  for t in ${TILES:-128 256 512}; do
    for f in 0 1; do
      echo "# HEAD $HEAD QSC_CTILE=$t QSC_FIN=$f" > $G/c2_t${t}_f${f}.log
      QSC_CTILE=$t QSC_FIN=$f timeout -k 10 200 python bench.py --config c2 --cpu-baseline 0 >> $G/c2_t${t}_f${f}.log 2>&1 || { tail -3 $G/c2_t${t}_f${f}.log; exit 1; }
      faulted $G/c2_t${t}_f${f}.log && exit 99
      summ $G/c2_t${t}_f${f}.log "c2 tile $t fin $f"
    done
  done
fi
if [ -z "$SKIP_C4" ]; then
  echo "# HEAD $HEAD" > $G/rehearsal/rehearse_n8_c4_kslab_strong.log
  QSC_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 8 --scaling strong --config c4 --shard kslab >> $G/rehearsal/rehearse_n8_c4_kslab_strong.log 2>&1 || { tail -5 $G/rehearsal/rehearse_n8_c4_kslab_strong.log; exit 1; }
  faulted $G/rehearsal/rehearse_n8_c4_kslab_strong.log && exit 99
  tail -1 $G/rehearsal/rehearse_n8_c4_kslab_strong.log | cut -c1-400
fi
if [ -z "$SKIP_C5" ]; then
  echo "# HEAD $HEAD" > $G/c5_explore.log
  timeout -k 10 500 python -u tools/c5_explore.py ${C5_ARGS} >> $G/c5_explore.log 2>&1 || { tail -5 $G/c5_explore.log; exit 1; }
  grep "^{" $G/c5_explore.log | cut -c1-300
fi
echo SESSION_DONE
