#!/bin/bash
# r04z: column dictionaries for the L = 8 SpMM (configs[4]'s CG) -- tree vs d24 (384 distinct panel
# rows per 1,024-item tile in 24 KB of LDS: 3 workgroups per CU) vs d12 (512-item tiles, 192 rows in
# 12 KB: 5 per CU) vs i8 (512-item tiles, no dictionary), alternating: the CG and its SpMM, then
# the L-wide SpMM shapes; parity of d24 and d12 on the GPU tests that run L = 8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04z; mkdir -p $OUT
for v in d24 d12; do
  MSPMV_LIB=$PWD/tools/lab/libmspmv_$v.so timeout -k 10 400 python -m pytest tests/test_gpu_spmv.py tests/test_gpu_cg.py tests/test_gpu_split_rows.py -m gpu -q -p no:cacheprovider -rf -x > $OUT/${v}_tests.log 2>&1
  rc=$?; echo "$v tests rc=$rc"; tail -3 $OUT/${v}_tests.log; [ $rc -le 1 ] || exit $rc
done
bash tools/lab/ab_libs.sh $OUT/cg 2 tools/lab/cgmulti_probe.py tree libmspmv_d24.so libmspmv_d12.so libmspmv_i8.so || exit 1
