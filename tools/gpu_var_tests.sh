#!/bin/bash
# GPU tests against a variant library, then A/B benches (tools/gpu_ab_env.sh)
#   LIB=variants/libqsc_x.so OUT=x ENVS="..." bash tools/gpu_var_tests.sh
G=gpurun_out/${OUT:-var}
mkdir -p $G
faulted() { grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU core dump" "$1"; }
QSC_LIB_PATH=$LIB timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $G/pytest_var.log 2>&1; rc=$?
tail -2 $G/pytest_var.log
faulted $G/pytest_var.log && { echo FAULT; exit 99; }
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $G/pytest_var.log | head; exit $rc; }
SKIP_TESTS=1 bash tools/gpu_ab_env.sh
