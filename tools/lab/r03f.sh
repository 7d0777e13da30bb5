#!/bin/bash
# r03f: k_spmm_blk X prefetch (tree) vs none; stamps of the prefetch build
cd "$(dirname "$0")/../.."
bash tools/lab/ab_libs.sh gpurun_out/r03f 2 tools/lab/spmm_cold_probe.py tree libmspmv_noxpf.so || exit 1
MSPMV_LIB=$PWD/tools/lab/libmspmv_stamps10.so timeout -k 10 200 python tools/lab/stamps_blk.py > gpurun_out/r03f/stamps.json 2>gpurun_out/r03f/stamps.err
