#!/bin/bash
# r05k: run-balanced node-block SpMV plan -- block tests, then pwtk / imperfect-FEM batches with the plan
# off / on (MSPMV_SPMV_RUNS), alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05k; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_blocks.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -4 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; exit 1; }
bash tools/lab/ab_env.sh $OUT/ab 2 "tools/lab/spmv_probe.py pwtk pwtk_perturbed" "MSPMV_SPMV_RUNS=0" "MSPMV_SPMV_RUNS=1" || exit 1
