#!/bin/bash
# r05d: column-slab SpMM ablation: LAB 1 no run sums, 2 panel rows from rows 0..127, 4 no panel loads
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05d; mkdir -p $OUT
bash tools/lab/ab_env.sh $OUT/ab 1 tools/lab/slabmm_probe.py "MSPMV_SPMM_SLAB=1 MSPMV_SLAB_LAB=2" "MSPMV_SPMM_SLAB=1 MSPMV_SLAB_LAB=4" \
  "MSPMV_SPMM_SLAB=1 MSPMV_SLAB_LAB=5" "MSPMV_SPMM_SLAB=1 MSPMV_SLAB_LAB=3" || exit 1
