#!/bin/bash
mkdir -p gpurun_out
QSC_LIB_PATH=variants/libqsc_stamps.so timeout -k 10 200 python tools/stamps_f.py
