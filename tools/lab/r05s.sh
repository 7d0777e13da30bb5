#!/bin/bash
# r05s: L-wide offset windows with LDS-staged runs of consecutive offsets (MSPMV_DIA_FORM=5): parity, then
# tiles vs form 1 vs form 5 (alternating).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05s; mkdir -p $OUT
MSPMV_DIA_FORM=5 timeout -k 10 600 python -u -m pytest tests/test_gpu_dia.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; exit 1; }
bash tools/lab/ab_env.sh $OUT/ab 2 tools/lab/dia_probe.py "MSPMV_DIA_SPMM=0" "MSPMV_DIA_SPMM=1 MSPMV_DIA_FORM=1" \
  "MSPMV_DIA_SPMM=1 MSPMV_DIA_FORM=5" || exit 1
