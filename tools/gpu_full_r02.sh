#!/bin/bash
# Round-2 measurement session: GPU tests + smoke + bench (with CPU leg) + rocprofv3 stats +
# FETCH/WRITE passes (tools/gpu_round.sh), then the SQ counter groups of the fused launch.
#   OUT=r02i bash tools/gpu_full_r02.sh
OUT=${OUT:-r02i}
OUT=$OUT bash tools/gpu_round.sh || exit $?
OUT=${OUT}_sq bash tools/pmc_sq2.sh || exit $?
echo FULL_DONE
