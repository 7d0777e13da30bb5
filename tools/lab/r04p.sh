#!/bin/bash
# r04p: the column-slab SpMV -- its parity tests, then tiles (MSPMV_SPMV_SLAB=0) vs slab (=1) on the
# scattered band, the power-law variant, cant and rma10, alternating; then what bounds the L-wide
# SpMM (g64: panel gathers folded onto 64 L1-resident rows; g0: no gather), one round.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04p; mkdir -p $OUT
timeout -k 10 300 python -m pytest tests/test_gpu_slab.py -m gpu -q -p no:cacheprovider -rf -x > $OUT/slab_tests.log 2>&1
rc=$?; echo "slab tests rc=$rc"; tail -30 $OUT/slab_tests.log; [ $rc -le 1 ] || exit $rc
export PROBE_SHAPES="scatter powerlaw cant"
for rep in 1 2; do
  for sw in 0 1; do
    MSPMV_SPMV_SLAB=$sw timeout -k 10 200 python3 tools/lab/spmv_probe.py > $OUT/spmv_slab${sw}_$rep.json 2>$OUT/spmv_slab${sw}_$rep.err || { echo "slab=$sw rc=$?"; tail -3 $OUT/spmv_slab${sw}_$rep.err; exit 1; }
    echo "slab=$sw $rep"; cat $OUT/spmv_slab${sw}_$rep.json
  done
done
bash tools/lab/ab_libs.sh $OUT/spmm 1 tools/lab/spmm_probe.py tree libmspmv_g64.so libmspmv_g0.so libmspmv_lg1.so libmspmv_lg2.so || exit 1
