#!/bin/bash
# r06kk: sliced-ELL first slices primed before the first slab of x is fetched (cur) vs the r06ii build (head),
# alternating twice: slab tests, the power-law leg and the scattered band.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06kk; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_slab.py tests/test_gpu_split_rows.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_slab.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest_slab.log | head -20; tail -5 $OUT/pytest_slab.log; exit 1; }
tail -1 $OUT/pytest_slab.log
for lib in cur head cur head; do
  if [ $lib = head ]; then E="MSPMV_LIB=$PWD/tools/lab/libmspmv_r06head.so"; else E="MSPMV_DUMMY=0"; fi
  env $E timeout -k 10 300 python bench.py --only spmv_shapes --no-cpu > $OUT/sh_${lib}.json 2>>$OUT/sh_${lib}.err || { echo "shapes rc=$?"; tail -3 $OUT/sh_${lib}.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/sh_${lib}.json'));print('$lib', [(k, d[k]['kernel'], d[k]['cold_kernel_ms'], d[k]['frac']) for k in ('cant','rma10','powerlaw')])"
  env $E timeout -k 10 300 python tools/lab/scatter_probe.py > $OUT/sc_${lib}.json 2>>$OUT/sc_${lib}.err || { echo "scatter rc=$?"; tail -3 $OUT/sc_${lib}.err; exit 1; }
  echo "$lib $(cat $OUT/sc_${lib}.json)"
done
echo done
