#!/bin/bash
# SQ counter groups of the fused launch with and without signed rows
OUT=sq_sr bash tools/pmc_sq2.sh || exit $?
QSC_SIGNED_ROWS=0 OUT=sq_nosr bash tools/pmc_sq2.sh || exit $?
echo SQ_AB_DONE
