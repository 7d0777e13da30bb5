#!/bin/bash
# r03r: grouped stream loads (W = 2 / 4 consecutive nonzeros per lane, lab builds g2 / g4) against the
# striped staging: SpMV parity tests per build, then the nlpkkt120-size SpMV and the spmv_shapes leg
# (cant, rma10, power-law), alternating builds, one process per run.
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03r; mkdir -p $OUT
for b in g2 g4; do
  MSPMV_LIB=$PWD/tools/lab/libmspmv_$b.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -m gpu tests/test_gpu_spmv.py tests/test_gpu_blocks.py > $OUT/tests_$b.log 2>&1; rc=$?
  echo "$b tests: $(tail -1 $OUT/tests_$b.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for b in tree g2 g4 g2tb; do
    case $b in tree) env="X=0";; g2tb) env="MSPMV_LIB=$PWD/tools/lab/libmspmv_g2.so MSPMV_SPMV_TB=64";; *) env="MSPMV_LIB=$PWD/tools/lab/libmspmv_$b.so";; esac
    env $env SWEEP_SHAPE=nlpkkt SWEEP_BATCH=1 timeout -k 10 200 python tools/spmv_sweep.py --child > $OUT/n.json 2>$OUT/n.err || { echo "$b nlpkkt failed"; tail -3 $OUT/n.err; exit 1; }
    env $env timeout -k 10 200 python bench.py --only spmv_shapes --no-cpu > $OUT/s.json 2>$OUT/s.err || { echo "$b shapes failed"; tail -3 $OUT/s.err; exit 1; }
    python3 - "$r" "$b" $OUT/n.json $OUT/s.json <<'PY'
import json, sys
n = json.load(open(sys.argv[3])); s = json.loads(open(sys.argv[4]).read().splitlines()[-1])
print(sys.argv[1], sys.argv[2], "nlpkkt cold", n["cold_kernel_us"], "us |",
      " ".join(f"{k} cold {s[k]['cold_kernel_ms']*1e3:.2f} us frac {s[k]['frac']}" for k in ("cant", "rma10", "powerlaw")))
PY
  done
done
