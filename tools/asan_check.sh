#!/bin/bash
# Host AddressSanitizer run of the C ABI: builds libqsc_hip_asan.so (host
# code sanitized; device code untouched) and runs the CPU tests that exercise host code paths
# (ABI argument checks, the host form of the list scheduler) against it with the clang ASan
# runtime preloaded.  CPU only: no GPU is touched.
#   bash tools/asan_check.sh [pytest args]
set -e
cd "$(dirname "$0")/.."
python -m quantized_spectrum_cartography_amd._build --asan
RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
LD_PRELOAD=$RT QSC_LIB_PATH=$PWD/quantized_spectrum_cartography_amd/libqsc_hip_asan.so \
  python -m pytest -q -x -m "not gpu" tests/test_sched_host.py tests/test_abi.py "$@"
