#!/bin/bash
# r04q (rerun as r04s): the column-slab SpMV after the plan-builder fix, stream prefetched two chunks ahead -- parity tests, then tiles vs slab on the
# scattered band and cant, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/${TAG:-r04q}; mkdir -p $OUT
timeout -k 10 300 python -m pytest tests/test_gpu_slab.py -m gpu -q -p no:cacheprovider -rf -x > $OUT/slab_tests.log 2>&1
rc=$?; echo "slab tests rc=$rc"; tail -15 $OUT/slab_tests.log; [ $rc -le 1 ] || exit $rc
export PROBE_SHAPES="scatter cant"
for rep in 1 2; do
  for sw in 0 1; do
    MSPMV_SPMV_SLAB=$sw timeout -k 10 200 python3 tools/lab/spmv_probe.py > $OUT/spmv_slab${sw}_$rep.json 2>$OUT/spmv_slab${sw}_$rep.err || { echo "slab=$sw rc=$?"; tail -3 $OUT/spmv_slab${sw}_$rep.err; exit 1; }
    echo "slab=$sw $rep"; cat $OUT/spmv_slab${sw}_$rep.json
  done
done
