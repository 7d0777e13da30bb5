#!/bin/bash
# r06gg: sliced-ELL short runs packed per lane only in the column-group plans (k_spmv_sell<.,true>), the band unpacked, vs the r06dd build (head),
# alternating: slab tests, the power-law leg and the scattered band.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06gg; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_slab.py tests/test_gpu_split_rows.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
  for lib in cur head; do
    if [ $lib = head ]; then E="MSPMV_LIB=$PWD/tools/lab/libmspmv_r06head.so"; else E="MSPMV_DUMMY=0"; fi
    env $E timeout -k 10 300 python bench.py --only spmv_shapes --no-cpu > $OUT/sh_${lib}_$i.json 2>$OUT/sh_${lib}_$i.err || { echo "shapes rc=$?"; tail -3 $OUT/sh_${lib}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/sh_${lib}_$i.json'));print('$lib', [(k, d[k]['kernel'], d[k]['cold_kernel_ms'], d[k]['frac']) for k in ('cant','rma10','powerlaw')])"
    env $E timeout -k 10 300 python tools/lab/scatter_probe.py > $OUT/sc_${lib}_$i.json 2>$OUT/sc_${lib}_$i.err || { echo "scatter rc=$?"; tail -3 $OUT/sc_${lib}_$i.err; exit 1; }
    echo "$lib $(cat $OUT/sc_${lib}_$i.json)"
  done
done
echo done
