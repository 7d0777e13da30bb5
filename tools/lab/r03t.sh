#!/bin/bash
# r03t: the committed tree (r03s: pair staging + one-wave skewed plans) and the paired-column node-block
# SpMV lab build (bp): parity, then the headline alternating tree / bp
cd "$(dirname "$0")/../.."
bash tools/lab/r03s.sh || exit $?
OUT=gpurun_out/r03t; mkdir -p $OUT
BP=$PWD/tools/lab/libmspmv_bp.so
MSPMV_LIB=$BP timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_blocks.py tests/test_gpu_fullsize.py -k "not cg" > $OUT/bp_tests.log 2>&1; rc=$?
tail -2 $OUT/bp_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for b in tree bp; do
  if [ $b = tree ]; then env="X=0"; else env="MSPMV_LIB=$BP"; fi
  env $env timeout -k 10 200 python bench.py --no-cg --no-extras --no-cpu > $OUT/h.json 2>$OUT/h.err || { tail -3 $OUT/h.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/h.json').read().splitlines()[-1]); print('$r $b', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['kernel'])"
done; done
