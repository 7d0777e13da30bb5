#!/bin/bash
# r03s: grouped (pair) stream loads by default + one-wave plans for skewed matrices -- SpMV/blocks/fullsize
# parity, then the spmv_shapes leg and the nlpkkt120-size SpMV
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03s; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fullsize.py tests/test_gpu_spmv.py tests/test_gpu_blocks.py > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --only spmv_shapes --no-cpu > $OUT/shapes.json 2>$OUT/shapes.err || exit 1
python3 -c "
import json; s=json.loads(open('$OUT/shapes.json').read().splitlines()[-1])
print(' '.join(f\"{k} {s[k]['kernel']} cold {s[k]['cold_kernel_ms']*1e3:.2f} us frac {s[k]['frac']}\" for k in ('cant','rma10','powerlaw')))"
SWEEP_SHAPE=nlpkkt SWEEP_BATCH=1 timeout -k 10 200 python tools/spmv_sweep.py --child > $OUT/n.json 2>$OUT/n.err || exit 1
cut -c1-400 $OUT/n.json
