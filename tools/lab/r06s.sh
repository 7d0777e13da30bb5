#!/bin/bash
# r06s: the one-group sliced-ELL plan as the line-bound default: slab / sell tests, smoke, and the bench lines
# (spmv_shapes for the power-law, the full bench for the scattered band).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06s; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_slab.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
for i in 1 2; do
  timeout -k 10 300 python tools/lab/scatter_probe.py > $OUT/scatter_$i.json 2>$OUT/scatter_$i.err || { echo "scatter rc=$?"; tail -3 $OUT/scatter_$i.err; exit 1; }
  cat $OUT/scatter_$i.json
done
echo done
