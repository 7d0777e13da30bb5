#!/bin/bash
# r04ak: L = 16 SpMM tile depth on the cant shape -- tree (32 items per lane group, 1,024-item tiles)
# vs i24 / i40 (768 / 1,280 items), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04ak; mkdir -p $OUT
bash tools/lab/ab_libs.sh $OUT/spmm 3 tools/lab/spmm_probe.py tree libmspmv_i24.so libmspmv_i40.so || exit 1
