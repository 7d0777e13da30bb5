#!/bin/bash
# r03aj: dictionary tiles with the pair staging's loads (lab build dp) -- parity, then cant / rma10 (dictionary
# tiles) and the scattered band, alternating tree / dp
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03aj; mkdir -p $OUT
DP=$PWD/tools/lab/libmspmv_dp.so
MSPMV_LIB=$DP timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_spmv.py tests/test_gpu_fullsize.py -k "not cg" > $OUT/dp_tests.log 2>&1; rc=$?
tail -1 $OUT/dp_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for b in tree dp; do
  if [ $b = tree ]; then env="X=0"; else env="MSPMV_LIB=$DP"; fi
  env $env timeout -k 10 200 python bench.py --only spmv_shapes --no-cpu > $OUT/s.json 2>$OUT/s.err || { tail -3 $OUT/s.err; exit 1; }
  env $env SWEEP_SHAPE=band SWEEP_BATCH=1 timeout -k 10 200 python tools/spmv_sweep.py --child > $OUT/b.json 2>$OUT/b.err || { tail -3 $OUT/b.err; exit 1; }
  python3 - "$r" "$b" $OUT/s.json $OUT/b.json <<'PY'
import json, sys
s = json.loads(open(sys.argv[3]).read().splitlines()[-1]); b = json.load(open(sys.argv[4]))
print(sys.argv[1], sys.argv[2], " ".join(f"{k} cold {s[k]['cold_kernel_ms']*1e3:.2f} hot {s[k]['hot_kernel_ms']*1e3:.2f} us" for k in ("cant", "rma10")),
      "| scattered band cold", b["cold_kernel_us"], "hot", b["hot_kernel_us"])
PY
done; done
