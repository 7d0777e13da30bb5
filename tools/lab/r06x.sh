#!/bin/bash
# r06x: sliced-ELL column groups of equal column counts (slabs from each block's first column): slab tests, then the
# power-law leg (54-55 us with whole-slab groups through r06v) and the scattered band.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06x; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_slab.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --only spmv_shapes --no-cpu > $OUT/sh_$i.json 2>$OUT/sh_$i.err || { echo "shapes rc=$?"; tail -3 $OUT/sh_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/sh_$i.json'));print([(k, d[k]['kernel'], d[k]['cold_kernel_ms'], d[k]['frac']) for k in ('cant','rma10','powerlaw')])"
done
timeout -k 10 300 python tools/lab/scatter_probe.py > $OUT/sc.json 2>$OUT/sc.err || { echo "scatter rc=$?"; tail -3 $OUT/sc.err; exit 1; }
cat $OUT/sc.json
echo done
