#!/bin/bash
# r05e: 4 stream register sets (panel 1 chunk ahead): full, and LAB 5 (no panel loads, no run sums)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05e; mkdir -p $OUT
bash tools/lab/ab_env.sh $OUT/ab 1 tools/lab/slabmm_probe.py "MSPMV_SPMM_SLAB=1" "MSPMV_SPMM_SLAB=1 MSPMV_SLAB_LAB=5" || exit 1
