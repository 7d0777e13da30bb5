#!/bin/bash
# r06t: one-group sliced-ELL (block-relative slabs) as the line-bound default: cant / rma10 / power-law legs and the
# scattered band with the default choice against MSPMV_SPMV_SLAB=0 (tiles), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06t; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for sw in def 0; do
    if [ $sw = def ]; then E="MSPMV_DUMMY=0"; else E="MSPMV_SPMV_SLAB=0"; fi
    env $E timeout -k 10 300 python bench.py --only spmv_shapes --no-cpu > $OUT/sh_${sw}_$i.json 2>$OUT/sh_${sw}_$i.err || { echo "shapes rc=$?"; tail -3 $OUT/sh_${sw}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/sh_${sw}_$i.json'));print('$sw', [(k, d[k]['kernel'], d[k]['cold_kernel_ms'], d[k]['frac']) for k in ('cant','rma10','powerlaw')])"
    env $E timeout -k 10 300 python tools/lab/scatter_probe.py > $OUT/sc_${sw}_$i.json 2>$OUT/sc_${sw}_$i.err || { echo "scatter rc=$?"; tail -3 $OUT/sc_${sw}_$i.err; exit 1; }
    echo "$sw $(cat $OUT/sc_${sw}_$i.json)"
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_slab.py -x -q --timeout 300 --timeout-method thread -k "not default_choice" > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
echo done
