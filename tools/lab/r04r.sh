#!/bin/bash
# r04r: column-slab SpMV geometry -- tree (512 threads, 4,096-column slabs, 2 blocks per CU) vs slab4
# (256 threads, 2,048-column slabs, 4 blocks per CU): parity tests of slab4, then both on the
# scattered band and cant (MSPMV_SPMV_SLAB=1), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04r; mkdir -p $OUT
MSPMV_LIB=$PWD/tools/lab/libmspmv_slab4.so timeout -k 10 300 python -m pytest tests/test_gpu_slab.py -m gpu -q -p no:cacheprovider -rf -k "not default" > $OUT/slab4_tests.log 2>&1
rc=$?; echo "slab4 tests rc=$rc"; tail -5 $OUT/slab4_tests.log; [ $rc -le 1 ] || exit $rc
export PROBE_SHAPES="scatter cant" MSPMV_SPMV_SLAB=1
bash tools/lab/ab_libs.sh $OUT/spmv 2 tools/lab/spmv_probe.py tree libmspmv_slab4.so || exit 1
