#!/bin/bash
# r05c: column-slab SpMM ablation (LAB bits: 1 no run sums, 2 panel rows from row 0) vs tiles
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05c; mkdir -p $OUT
bash tools/lab/ab_env.sh $OUT/ab 1 tools/lab/slabmm_probe.py "MSPMV_SPMM_SLAB=0" "MSPMV_SPMM_SLAB=1" \
  "MSPMV_SPMM_SLAB=1 MSPMV_SLAB_LAB=1" "MSPMV_SPMM_SLAB=1 MSPMV_SLAB_LAB=2" "MSPMV_SPMM_SLAB=1 MSPMV_SLAB_LAB=3" || exit 1
