#!/bin/bash
# r03am: tile size of the node-block plan (items per thread 6 / 7 / 8 / 16 -> 1536 .. 4096 merge items,
# ~4.7 .. 12.6 runs of 6 rows for the 8 half-wave slots of a k_spmv_blk workgroup) on the headline
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03am; mkdir -p $OUT
for r in 1 2; do for v in 8 16 7 6; do
  MSPMV_SPMV_IPT=$v timeout -k 10 200 python bench.py --no-cg --no-extras --no-cpu > $OUT/h.json 2>$OUT/h.err || { tail -3 $OUT/h.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/h.json').read().splitlines()[-1]); print('$r ipt=$v', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['kernel'])"
done; done
