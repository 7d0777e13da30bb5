#!/bin/bash
# r05n: run-balanced plan at 256 threads (8 run slots) vs 512 threads (16 run slots, MSPMV_RUN_WIDE=1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05n; mkdir -p $OUT
MSPMV_RUN_WIDE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_blocks.py -x -q --timeout 300 --timeout-method thread -k "run_plan or mixed or perturbed_full or full_pwtk" > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; exit 1; }
bash tools/lab/ab_env.sh $OUT/spmv 3 "tools/lab/spmv_probe.py pwtk pwtk_perturbed" "MSPMV_RUN_WIDE=0" "MSPMV_RUN_WIDE=1" || exit 1
