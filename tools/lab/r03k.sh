#!/bin/bash
# r03k: read+write pass shapes (tools/rw_probe) and the SpMV tile order with K streams per XCD
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03k; mkdir -p $OUT
timeout -k 10 120 tools/rw_probe > $OUT/rw_probe.txt 2>&1 || exit 1
cat $OUT/rw_probe.txt
for r in 1 2; do
for K in 1 2 4 8 32; do
  for shape in nlpkkt fem; do
    B=4; [ $shape = nlpkkt ] && B=1
    MSPMV_TILE_STREAMS=$K SWEEP_SHAPE=$shape SWEEP_BATCH=$B timeout -k 10 200 python tools/spmv_sweep.py --child > $OUT/k${K}_${shape}_$r.json 2>$OUT/k${K}_${shape}_$r.err || exit 1
    echo "K=$K $shape $(cat $OUT/k${K}_${shape}_$r.json)"
  done
done
done
