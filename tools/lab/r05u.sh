#!/bin/bash
# r05u: L = 1 offset-window ablations (MSPMV_DIA_FORM1 3: no x loads, 4: no panel loads; timing only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05u; mkdir -p $OUT
bash tools/lab/ab_env.sh $OUT/ab 2 tools/lab/dia_probe.py "MSPMV_DIA_FORM1=0" "MSPMV_DIA_FORM1=3" "MSPMV_DIA_FORM1=4" || exit 1
