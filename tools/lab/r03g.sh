#!/bin/bash
# r03g: k_spmm_blk straight-line passes (tree: PB 2, 82 VGPRs) vs the r03a kernel (old) and register-bound variants
cd "$(dirname "$0")/../.."
bash tools/lab/ab_libs.sh gpurun_out/r03g 2 tools/lab/spmm_cold_probe.py tree libmspmv_old.so libmspmv_w8f.so libmspmv_pb1.so libmspmv_pb1w8.so
