#!/bin/bash
# r06o: the sliced-ELL SpMV cut for two 512-thread blocks per CU (7,168-column slabs, MSPMV_SELL_CFG=3) against one
# 1,024-thread block per CU (14,336 columns): parity under cfg 3, then the power-law leg alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06o; mkdir -p $OUT
export TMPDIR=/tmp
MSPMV_SELL_CFG=3 timeout -k 10 900 python -u -m pytest tests/test_gpu_slab.py "tests/test_gpu_fullsize.py::test_spmv_full_size" -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
  for c in 2 3; do
    MSPMV_SELL_CFG=$c timeout -k 10 300 python bench.py --only spmv_shapes --no-cpu > $OUT/sh_${c}_$i.json 2>$OUT/sh_${c}_$i.err || { echo "shapes rc=$?"; tail -3 $OUT/sh_${c}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/sh_${c}_$i.json'));p=d['powerlaw'];print('cfg=$c', p['kernel'], p['cold_kernel_ms'], p['hot_kernel_ms'], p['frac'])"
  done
done
echo done
