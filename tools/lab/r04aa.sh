#!/bin/bash
# r04aa: L = 16 SpMM tile depth -- tree (16 items per lane group: 512-item tiles) vs i32 (1,024-item
# tiles: half the tile start-ups, 6 workgroups per CU), alternating; parity of i32 on the SpMM tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04aa; mkdir -p $OUT
MSPMV_LIB=$PWD/tools/lab/libmspmv_i32.so timeout -k 10 300 python -m pytest tests/test_gpu_spmv.py tests/test_gpu_split_rows.py -m gpu -q -p no:cacheprovider -rf > $OUT/i32_tests.log 2>&1
rc=$?; echo "i32 tests rc=$rc"; tail -4 $OUT/i32_tests.log; [ $rc -le 1 ] || exit $rc
bash tools/lab/ab_libs.sh $OUT/spmm 2 tools/lab/spmm_probe.py tree libmspmv_i32.so || exit 1
