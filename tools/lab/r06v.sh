#!/bin/bash
# r06v: split-row tickets in the drained-store form only; the skewed SpMV on one-wave tiles (MSPMV_SPMV_SLAB=0) with
# this build and with the round-5 library, alternating; split-row tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06v; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_split_rows.py tests/test_gpu_spmv.py tests/test_gpu_slab.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
  for lib in cur r05; do
    if [ $lib = r05 ]; then E="MSPMV_LIB=$PWD/tools/lab/libmspmv_r05.so"; else E="MSPMV_DUMMY=0"; fi
    env $E MSPMV_SPMV_SLAB=0 timeout -k 10 300 python bench.py --only spmv_shapes --no-cpu > $OUT/sh_${lib}_$i.json 2>$OUT/sh_${lib}_$i.err || { echo "shapes rc=$?"; tail -3 $OUT/sh_${lib}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/sh_${lib}_$i.json'));print('$lib', [(k, d[k]['kernel'], d[k]['cold_kernel_ms'], d[k]['frac']) for k in ('cant','rma10','powerlaw')])"
  done
done
echo done
