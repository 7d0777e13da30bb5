#!/bin/bash
# r05i: resident CG tests (both forms, stall fallback) and configs[3] classic vs single-reduction A/B
# single-reduction resident CG, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05i; mkdir -p $OUT
true
true
timeout -k 10 600 python -u -m pytest tests/test_gpu_cg_resident.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -4 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; exit 1; }
bash tools/lab/ab_env.sh $OUT/ab 2 tools/lab/cg1_probe.py "MSPMV_CG_RESIDENT_FORM=classic" "MSPMV_CG_RESIDENT_FORM=single_reduction" || exit 1
