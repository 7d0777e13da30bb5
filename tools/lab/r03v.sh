#!/bin/bash
# r03v: node-block SpMM with the run's values loaded as column pairs (lab build sv2) -- parity, then the
# spmm16 leg (cant, pwtk, cold + hot) alternating tree / sv2
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03v; mkdir -p $OUT
SV2=$PWD/tools/lab/libmspmv_sv2.so
MSPMV_LIB=$SV2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_blocks.py tests/test_gpu_fullsize.py -k "not cg" > $OUT/sv2_tests.log 2>&1; rc=$?
tail -1 $OUT/sv2_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for b in tree sv2; do
  if [ $b = tree ]; then env="X=0"; else env="MSPMV_LIB=$SV2"; fi
  env $env timeout -k 10 200 python bench.py --only spmm16 --no-cpu > $OUT/s.json 2>$OUT/s.err || { tail -3 $OUT/s.err; exit 1; }
  python3 -c "
import json; s=json.loads(open('$OUT/s.json').read().splitlines()[-1])
print('$r $b', ' '.join(f\"{k} cold {s[k]['cold_kernel_ms']*1e3:.2f} hot {s[k]['hot_kernel_ms']*1e3:.2f} us frac {s[k]['frac']}\" for k in ('cant','pwtk')))"
done; done
