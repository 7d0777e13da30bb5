#!/bin/bash
# r03aa: one contiguous slice per workgroup in the CG streaming passes (lab build vs) -- CG parity, then the multi-RHS
# CG leg (nlpkkt120 size, L = 8: its SpMM is k_spmm_tile<8,16,...>) alternating tree / vs
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03aa; mkdir -p $OUT
VS=$PWD/tools/lab/libmspmv_vs.so
MSPMV_LIB=$VS timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_cg.py tests/test_gpu_dist.py tests/test_spai.py tests/test_ic0.py > $OUT/vs_tests.log 2>&1; rc=$?
tail -1 $OUT/vs_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for b in tree vs; do
  if [ $b = tree ]; then env="X=0"; else env="MSPMV_LIB=$VS"; fi
  env $env timeout -k 10 200 python bench.py --only cg_multi --no-cpu > $OUT/c.json 2>$OUT/c.err || { tail -3 $OUT/c.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/c.json').read().splitlines()[-1])
print('$r $b cg_multi', d['ms_per_iter'], 'ms/iter frac', d['roofline_frac'], '| nlpkkt spmv', d['spmv_nlpkkt120_size']['kernel_ms'])"
done; done
