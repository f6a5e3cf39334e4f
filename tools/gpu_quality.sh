#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/quality_c5.py "$@" > gpurun_out/quality.json 2> gpurun_out/quality.err
rc=$?; cat gpurun_out/quality.json; tail -5 gpurun_out/quality.err; exit $rc
