#!/bin/bash
# r06y: sliced-ELL power-law plan with 6,143-row blocks, 12,288-column slabs and 5 column groups (MSPMV_SELL_CFG=3
# MSPMV_SLAB_GROUPS=5: the busiest block 54.4 K items instead of 64.9 K) against the default (4,095 rows, 14,336
# columns, 4 groups); parity of the default choice under cfg 3, then the power-law leg alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06y; mkdir -p $OUT
export TMPDIR=/tmp
MSPMV_SELL_CFG=3 MSPMV_SLAB_GROUPS=5 timeout -k 10 600 python -u -m pytest tests/test_gpu_slab.py -k default_choice -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2 3; do
  for v in base new; do
    if [ $v = new ]; then E="MSPMV_SELL_CFG=3 MSPMV_SLAB_GROUPS=5"; else E="MSPMV_DUMMY=0"; fi
    env $E timeout -k 10 300 python bench.py --only spmv_shapes --no-cpu > $OUT/sh_${v}_$i.json 2>$OUT/sh_${v}_$i.err || { echo "shapes rc=$?"; tail -3 $OUT/sh_${v}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/sh_${v}_$i.json'));p=d['powerlaw'];print('$v', p['kernel'], p['cold_kernel_ms'], p['hot_kernel_ms'], p['frac'])"
  done
done
echo done
