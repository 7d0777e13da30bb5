#!/bin/bash
# r05t: offset windows -- L = 1 unroll 8 / 16 / 32 (MSPMV_DIA_FORM1 0 / 1 / 2) paired with the L-wide LDS-run
# form at 4 / 5 / 6 waves per SIMD (MSPMV_DIA_FORM 5 / 6 / 7), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05t; mkdir -p $OUT
bash tools/lab/ab_env.sh $OUT/ab 2 tools/lab/dia_probe.py "MSPMV_DIA_SPMM=1 MSPMV_DIA_FORM=5 MSPMV_DIA_FORM1=0" \
  "MSPMV_DIA_SPMM=1 MSPMV_DIA_FORM=6 MSPMV_DIA_FORM1=1" "MSPMV_DIA_SPMM=1 MSPMV_DIA_FORM=7 MSPMV_DIA_FORM1=2" || exit 1
