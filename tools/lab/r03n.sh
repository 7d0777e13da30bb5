#!/bin/bash
# r03n: the dot-mode SpMM with its x.(Ax) taken in a tail pass (kSpmmDotTail, 70 VGPRs at L = 8 like
# the plain SpMM) -- CG/SPAI parity tests, then the split CG's p.Ap: separate pass vs the SpMM's dot mode
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03n; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_cg.py tests/test_spai.py tests/test_gpu_dist.py > $OUT/tests.log 2>&1; rc=$?
tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in pass fused; do
  MSPMV_CG_DOT=$v timeout -k 10 200 python bench.py --only cg_multi --no-cpu > $OUT/cgm_${v}_$i.json 2>$OUT/cgm_${v}_$i.err || exit 1
  echo "$v $i $(cut -c1-400 $OUT/cgm_${v}_$i.json | sed 's/.*"iterations"/"iterations"/')"
done; done
