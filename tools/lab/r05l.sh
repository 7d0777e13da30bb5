#!/bin/bash
# r05l: run-balanced plan caps: items per tile (% of the merge-path tile) and run chunks per tile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05l; mkdir -p $OUT
bash tools/lab/ab_env.sh $OUT/ab 2 "tools/lab/spmv_probe.py pwtk pwtk_perturbed" "MSPMV_SPMV_RUNS=0" \
  "MSPMV_RUN_CAP_PCT=112" "MSPMV_RUN_CAP_PCT=125" "MSPMV_RUN_CAP_PCT=150" "MSPMV_RUN_CAP_PCT=200" \
  "MSPMV_RUN_CAP_CHUNKS=7" "MSPMV_RUN_CAP_PCT=150 MSPMV_RUN_CAP_CHUNKS=7" || exit 1
