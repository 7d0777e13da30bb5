#!/bin/bash
# r03y: tile depth on the one-wave plans of the skewed variant (items per thread 4 / 6 / 8 / 16; the
# knob sets every plan's depth, so only the power-law line is read), and the walk/group cost budget
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03y; mkdir -p $OUT
for r in 1 2; do
  for v in "X=0" "MSPMV_SPMV_IPT=4" "MSPMV_SPMV_IPT=6" "MSPMV_SPMV_IPT=16" "MSPMV_SPMV_RG_COST=0" "MSPMV_SPMV_RG_COST=96"; do
    env $v timeout -k 10 200 python bench.py --only spmv_shapes --no-cpu > $OUT/s.json 2>$OUT/s.err || { echo "$v failed"; tail -3 $OUT/s.err; exit 1; }
    python3 -c "
import json; s=json.loads(open('$OUT/s.json').read().splitlines()[-1])
print('$r $v', ' '.join(f\"{k} {s[k]['kernel']} {s[k]['cold_kernel_ms']*1e3:.2f} us\" for k in ('cant','rma10','powerlaw')))"
  done
done
