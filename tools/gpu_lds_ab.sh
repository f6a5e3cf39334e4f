#!/bin/bash
# LDS counters of the fused launch for the default library and a variant ($LIB)
G3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
OUT=lds_a bash tools/gpu_pmc.sh "$G3" || exit $?
QSC_LIB_PATH=$LIB OUT=lds_b bash tools/gpu_pmc.sh "$G3" || exit $?
