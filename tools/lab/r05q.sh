#!/bin/bash
# r05q: the L-wide offset-window kernel's lab forms (MSPMV_DIA_FORM 0-4), alternating, and the tiles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05q; mkdir -p $OUT
bash tools/lab/ab_env.sh $OUT/ab 2 tools/lab/dia_probe.py "MSPMV_DIA=0" "MSPMV_DIA_FORM=0" "MSPMV_DIA_FORM=1" \
  "MSPMV_DIA_FORM=2" "MSPMV_DIA_FORM=3" "MSPMV_DIA_FORM=4" || exit 1
