#!/bin/bash
# r03af: pair staging with one 16-B x load for consecutive column pairs (lab build xp) -- parity, then the
# nlpkkt120-size SpMV and the spmv_shapes leg alternating tree / xp
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03af; mkdir -p $OUT
XP=$PWD/tools/lab/libmspmv_xp.so
MSPMV_LIB=$XP timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_spmv.py tests/test_gpu_fullsize.py -k "not cg" > $OUT/xp_tests.log 2>&1; rc=$?
tail -1 $OUT/xp_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for b in tree xp; do
  if [ $b = tree ]; then env="X=0"; else env="MSPMV_LIB=$XP"; fi
  env $env SWEEP_SHAPE=nlpkkt SWEEP_BATCH=1 timeout -k 10 200 python tools/spmv_sweep.py --child > $OUT/n.json 2>$OUT/n.err || { tail -3 $OUT/n.err; exit 1; }
  env $env timeout -k 10 200 python bench.py --only spmv_shapes --no-cpu > $OUT/s.json 2>$OUT/s.err || { tail -3 $OUT/s.err; exit 1; }
  python3 - "$r" "$b" $OUT/n.json $OUT/s.json <<'PY'
import json, sys
n = json.load(open(sys.argv[3])); s = json.loads(open(sys.argv[4]).read().splitlines()[-1])
print(sys.argv[1], sys.argv[2], "nlpkkt cold", n["cold_kernel_us"], "us |",
      " ".join(f"{k} cold {s[k]['cold_kernel_ms']*1e3:.2f} us" for k in ("cant", "rma10", "powerlaw")))
PY
done; done
