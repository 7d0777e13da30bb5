#!/bin/bash
# r03c: k_spmm_blk variants (guarded mul+add vs FMA; gathers in flight per round) on configs[2] shapes
cd "$(dirname "$0")/../.."
bash tools/lab/ab_libs.sh gpurun_out/r03c 2 tools/lab/spmm_cold_probe.py tree libmspmv_nofma.so libmspmv_pb4.so libmspmv_pb8.so libmspmv_pb8w6.so
