#!/bin/bash
# r06hh: the packed sliced-ELL build (short runs packed per lane in the column-group plans only) against the r06dd
# build (head) on the power-law leg and the scattered band, then the final evidence session on this tree
# (smoke, every GPU test, bench, kernel traces, PMC passes, per-leg profiles).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06hh; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_slab.py tests/test_gpu_split_rows.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_slab.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest_slab.log | head -20; tail -5 $OUT/pytest_slab.log; exit 1; }
tail -1 $OUT/pytest_slab.log
for lib in cur head; do
  if [ $lib = head ]; then E="MSPMV_LIB=$PWD/tools/lab/libmspmv_r06head.so"; else E="MSPMV_DUMMY=0"; fi
  env $E timeout -k 10 300 python bench.py --only spmv_shapes --no-cpu > $OUT/sh_${lib}.json 2>$OUT/sh_${lib}.err || { echo "shapes rc=$?"; tail -3 $OUT/sh_${lib}.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/sh_${lib}.json'));print('$lib', [(k, d[k]['kernel'], d[k]['cold_kernel_ms'], d[k]['frac']) for k in ('cant','rma10','powerlaw')])"
  env $E timeout -k 10 300 python tools/lab/scatter_probe.py > $OUT/sc_${lib}.json 2>$OUT/sc_${lib}.err || { echo "scatter rc=$?"; tail -3 $OUT/sc_${lib}.err; exit 1; }
  echo "$lib $(cat $OUT/sc_${lib}.json)"
done
bash tools/gpu_session.sh r06hh smoke tests bench prof pmc legs:spmm16,spmv_shapes,cg_single,cg_multi
