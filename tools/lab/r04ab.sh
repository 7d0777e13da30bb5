#!/bin/bash
# r04ab: L-wide SpMM tile depth -- tree (L = 16: 16 items per lane group) vs i32 / i48 / i64 (L = 16:
# 32 / 48 / 64; dictionary budget 16 KB) vs j32 (L = 8 and 16: 32), alternating; the SpMM and CG
# parity tests on i32 and i48.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04ab; mkdir -p $OUT
for v in i32 i48; do
  MSPMV_LIB=$PWD/tools/lab/libmspmv_$v.so timeout -k 10 400 python -m pytest tests/test_gpu_spmv.py tests/test_gpu_split_rows.py tests/test_gpu_cg.py tests/test_gpu_blocks.py -m gpu -q -p no:cacheprovider -rf > $OUT/${v}_tests.log 2>&1
  rc=$?; echo "$v tests rc=$rc"; tail -3 $OUT/${v}_tests.log; [ $rc -le 1 ] || exit $rc
done
bash tools/lab/ab_libs.sh $OUT/spmm 2 tools/lab/spmm_probe.py tree libmspmv_i32.so libmspmv_i48.so libmspmv_i64.so libmspmv_j32.so || exit 1
