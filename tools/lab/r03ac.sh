#!/bin/bash
# r03ac: the single-RHS plan's generation stretch (longer tiles, some rows split -> carry fix-up) on vs
# off, now that the fix-up is timed: spmv_shapes leg (cant, rma10) and the CG single leg, alternating
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03ac; mkdir -p $OUT
for r in 1 2; do for v in 1 0; do
  MSPMV_SPMV_STRETCH=$v timeout -k 10 200 python bench.py --only spmv_shapes --no-cpu > $OUT/s.json 2>$OUT/s.err || { tail -3 $OUT/s.err; exit 1; }
  python3 -c "
import json; s=json.loads(open('$OUT/s.json').read().splitlines()[-1])
print('$r stretch=$v', ' '.join(f\"{k} cold {s[k]['cold_kernel_ms']*1e3:.2f} hot {s[k]['hot_kernel_ms']*1e3:.2f} us\" for k in ('cant','rma10','powerlaw')))"
done; done
