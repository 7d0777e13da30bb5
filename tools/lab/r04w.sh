#!/bin/bash
# r04w: the column-slab SpMV's run sums -- tree vs ds (yacc += as an LDS atomic add: one writer per
# row and chunk, so the same sum, without the read round trip) vs cm (lanes per run from a rounds x
# steps cost model instead of 4 G >= mean) vs both, forced on, scattered band and cant; then the
# slab tests on the "both" build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04w; mkdir -p $OUT
MSPMV_LIB=$PWD/tools/lab/libmspmv_both.so timeout -k 10 300 python -m pytest tests/test_gpu_slab.py -m gpu -q -p no:cacheprovider -rf > $OUT/both_tests.log 2>&1
rc=$?; echo "both tests rc=$rc"; tail -3 $OUT/both_tests.log; [ $rc -le 1 ] || exit $rc
export PROBE_SHAPES="scatter cant" MSPMV_SPMV_SLAB=1
bash tools/lab/ab_libs.sh $OUT/spmv 2 tools/lab/spmv_probe.py tree libmspmv_ds.so libmspmv_cm.so libmspmv_both.so || exit 1
