#!/bin/bash
# r06p: the pipelined single CG's update grid (MSPMV_CG1_BLOCKS cap 1024 / 512 / 256): every SpMV workgroup and every
# update workgroup sums the other kernel's partials, so fewer update blocks mean fewer partials loaded by each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06p; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for nb in 1024 512 256; do
    MSPMV_CG_RESIDENT=0 MSPMV_CG1_BLOCKS=$nb timeout -k 10 300 python tools/lab/cg_large_probe.py > $OUT/cgl_${nb}_$i.json 2>$OUT/cgl_${nb}_$i.err || { echo "cgl rc=$?"; tail -3 $OUT/cgl_${nb}_$i.err; exit 1; }
    echo "nb=$nb $(cat $OUT/cgl_${nb}_$i.json)"
  done
done
MSPMV_CG_RESIDENT=0 MSPMV_CG1_BLOCKS=256 timeout -k 10 600 python -u -m pytest tests/test_gpu_cg.py -k pipelined -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
echo done
