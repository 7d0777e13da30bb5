#!/bin/bash
# r04u: column-slab geometry -- tree (4,096-column slabs, 2 blocks per CU) vs slab3 (2,048-column
# slabs, 1,023 rows, 3 blocks per CU), forced on, scattered band and cant, alternating; then the slab
# tests (default choice now on).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04u; mkdir -p $OUT
timeout -k 10 300 python -m pytest tests/test_gpu_slab.py -m gpu -q -p no:cacheprovider -rf > $OUT/slab_tests.log 2>&1
rc=$?; echo "slab tests rc=$rc"; tail -4 $OUT/slab_tests.log; [ $rc -le 1 ] || exit $rc
MSPMV_LIB=$PWD/tools/lab/libmspmv_slab3.so timeout -k 10 300 python -m pytest tests/test_gpu_slab.py -m gpu -q -p no:cacheprovider -rf -k "not default" > $OUT/slab3_tests.log 2>&1
rc=$?; echo "slab3 tests rc=$rc"; tail -3 $OUT/slab3_tests.log; [ $rc -le 1 ] || exit $rc
export PROBE_SHAPES="scatter cant" MSPMV_SPMV_SLAB=1
bash tools/lab/ab_libs.sh $OUT/spmv 2 tools/lab/spmv_probe.py tree libmspmv_slab3.so || exit 1
