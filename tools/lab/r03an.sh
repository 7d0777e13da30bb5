#!/bin/bash
# r03an: a wide node-block plan for the plain SpMV (MSPMV_BLK_TILE merge items per tile: up to two rounds
# of the 8 half-wave run slots) -- parity at 3072, then the headline at 0 (off) / 2560 / 3072 / 4096
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03an; mkdir -p $OUT
MSPMV_BLK_TILE=3072 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_blocks.py tests/test_gpu_fullsize.py -k "not cg" > $OUT/tests.log 2>&1; rc=$?
tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in 0 2560 3072 4096; do
  MSPMV_BLK_TILE=$v timeout -k 10 200 python bench.py --no-cg --no-extras --no-cpu > $OUT/h.json 2>$OUT/h.err || { tail -3 $OUT/h.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/h.json').read().splitlines()[-1]); print('$r blk_tile=$v', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['kernel'])"
done; done
