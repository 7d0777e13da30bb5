#!/bin/bash
# r03ai: row ends issued with the stream (MSPMV_SPMV_EARLY_RE=1) on the other single-RHS tile shapes
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03ai; mkdir -p $OUT
for r in 1 2; do for v in 0 1; do
  MSPMV_SPMV_EARLY_RE=$v timeout -k 10 200 python bench.py --only spmv_shapes --no-cpu > $OUT/s.json 2>$OUT/s.err || { tail -3 $OUT/s.err; exit 1; }
  python3 -c "
import json; s=json.loads(open('$OUT/s.json').read().splitlines()[-1])
print('$r early_re=$v', ' '.join(f\"{k} cold {s[k]['cold_kernel_ms']*1e3:.2f} hot {s[k]['hot_kernel_ms']*1e3:.2f} us\" for k in ('cant','rma10','powerlaw')))"
  MSPMV_SPMV_EARLY_RE=$v MSPMV_CG_RESIDENT=0 timeout -k 10 200 python bench.py --only cg_single --no-cpu > $OUT/c.json 2>$OUT/c.err || { tail -3 $OUT/c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c.json').read().splitlines()[-1]); print('$r early_re=$v cg_single (pipelined form)', d['us_per_iter'])"
done; done
