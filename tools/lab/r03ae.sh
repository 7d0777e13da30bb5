#!/bin/bash
# r03ae: node-block SpMV pairs gathering x once per consecutive column pair (plan-checked) vs per column
# (MSPMV_BLK_PAIRGATHER=0): parity, then the headline alternating
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03ae; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_blocks.py tests/test_gpu_fullsize.py tests/test_gpu_spmv.py tests/test_gpu_dist.py -k "not cg_multi" > $OUT/tests.log 2>&1; rc=$?
tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -3 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for r in 1 2 3; do for v in 1 0; do
  MSPMV_BLK_PAIRGATHER=$v timeout -k 10 200 python bench.py --no-cg --no-extras --no-cpu > $OUT/h.json 2>$OUT/h.err || { tail -3 $OUT/h.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/h.json').read().splitlines()[-1]); print('$r pairgather=$v', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done; done
