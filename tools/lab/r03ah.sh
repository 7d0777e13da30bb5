#!/bin/bash
# r03ah: tile depth (items per thread) on the nlpkkt120-size SpMV with the pair staging, alternating
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03ah; mkdir -p $OUT
export SWEEP_SHAPE=nlpkkt SWEEP_BATCH=1
for r in 1 2; do
  for v in "X=0" "MSPMV_SPMV_IPT=6" "MSPMV_SPMV_IPT=7" "MSPMV_SPMV_IPT=16" "MSPMV_SPMV_EARLY_RE=1"; do
    env $v timeout -k 10 200 python tools/spmv_sweep.py --child > $OUT/run.json 2>$OUT/run.err || { echo "$v failed"; tail -3 $OUT/run.err; exit 1; }
    echo "$r $v $(python3 -c "import json; d=json.load(open('$OUT/run.json')); print(d['cold_kernel_us'], d['hot_kernel_us'])")"
  done
done
