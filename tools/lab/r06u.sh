#!/bin/bash
# r06u: split-row tickets released only for rows of <= 8 carries; band sell threshold at the slab blocks' bar.
# Tests (slab, split rows, spmv, faults), smoke, then the skewed SpMV on one-wave tiles (MSPMV_SPMV_SLAB=0) and the
# default legs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06u; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_slab.py tests/test_gpu_split_rows.py tests/test_gpu_spmv.py tests/test_gpu_faults.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for i in 1 2; do
  for sw in def 0; do
    if [ $sw = def ]; then E="MSPMV_DUMMY=0"; else E="MSPMV_SPMV_SLAB=0"; fi
    env $E timeout -k 10 300 python bench.py --only spmv_shapes --no-cpu > $OUT/sh_${sw}_$i.json 2>$OUT/sh_${sw}_$i.err || { echo "shapes rc=$?"; tail -3 $OUT/sh_${sw}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/sh_${sw}_$i.json'));print('$sw', [(k, d[k]['kernel'], d[k]['cold_kernel_ms'], d[k]['frac']) for k in ('cant','rma10','powerlaw')])"
  done
  timeout -k 10 300 python tools/lab/scatter_probe.py > $OUT/sc_$i.json 2>$OUT/sc_$i.err || { echo "scatter rc=$?"; tail -3 $OUT/sc_$i.err; exit 1; }
  cat $OUT/sc_$i.json
done
echo done
