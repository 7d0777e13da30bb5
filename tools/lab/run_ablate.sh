#!/bin/bash
# GPU side of the ablation lab: one sweep child per library variant, then the stream ceiling.
cd "$(dirname "$0")/../.."
for n in "$@"; do
  MSPMV_LIB=$PWD/tools/lab/libmspmv_abl$n.so MSPMV_SPMV_IPT=8 MSPMV_SPMV_NT=1 timeout -k 10 120 \
      python tools/spmv_sweep.py --child > gpurun_out/abl_$n.json 2>gpurun_out/abl_$n.err || { echo "abl $n rc=$?"; exit 1; }
  echo "abl $n $(cat gpurun_out/abl_$n.json)"
done
