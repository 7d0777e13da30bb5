#!/bin/bash
# r03al: the nlpkkt120-size SpMV (pair staging, row ends with the stream) under the remaining knobs:
# regular (not nontemporal) matrix loads, 2 / 4 side-by-side tile streams per XCD, row-group budgets
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03al; mkdir -p $OUT
export SWEEP_SHAPE=nlpkkt SWEEP_BATCH=1
for r in 1 2; do
  for v in "X=0" "MSPMV_SPMV_NT=0" "MSPMV_TILE_STREAMS=2" "MSPMV_TILE_STREAMS=4" "MSPMV_SPMV_RG_COST=24" "MSPMV_SPMV_RG_COST=96"; do
    env $v timeout -k 10 200 python tools/spmv_sweep.py --child > $OUT/run.json 2>$OUT/run.err || { echo "$v failed"; tail -3 $OUT/run.err; exit 1; }
    echo "$r $v $(python3 -c "import json; d=json.load(open('$OUT/run.json')); print(d['cold_kernel_us'], d['hot_kernel_us'], d['modes'][:4])")"
  done
done
