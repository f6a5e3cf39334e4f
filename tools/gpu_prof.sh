#!/bin/bash
# Counter collection for the fused kernels (separate --pmc passes; no tracing domains mixed in).
#   bash tools/gpu_prof.sh [extra prof_passes.py args]
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "spass|cpass|cfinish" -d $R/gpurun_out/pmc/$name -o run --output-format csv -- python3 $R/tools/prof_passes.py --iters 10 $PROF_ARGS > $R/gpurun_out/pmc/$name.log 2>&1 || { echo "FAIL $name rc=$?"; tail -20 $R/gpurun_out/pmc/$name.log; exit 1; }
  echo "ok $name"
}
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT
run sq2 SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
run grbm GRBM_GUI_ACTIVE GRBM_COUNT
run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
