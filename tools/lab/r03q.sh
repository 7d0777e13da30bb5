#!/bin/bash
# r03q: which resource bounds the generic tile SpMV on the nlpkkt120-size 27-point matrix (1.2 GB per
# launch)?  Knob sensitivity, alternating, one process per run: default, int32 columns (+2 B/nnz, same
# instruction count), one-wave tiles, row ends with the stream, merge walk everywhere, 7 items/thread.
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03q; mkdir -p $OUT
export SWEEP_SHAPE=nlpkkt SWEEP_BATCH=1
for r in 1 2; do
  for v in "X=0" "MSPMV_SPMV_C16=0" "MSPMV_SPMV_TB=64" "MSPMV_SPMV_EARLY_RE=1" "MSPMV_SPMV_RG_COST=0" "MSPMV_SPMV_IPT=7"; do
    env $v timeout -k 10 200 python tools/spmv_sweep.py --child > $OUT/run.json 2>$OUT/run.err || { echo "$v failed"; tail -3 $OUT/run.err; exit 1; }
    echo "$r $v $(cat $OUT/run.json)"
  done
done
