#!/bin/bash
# r05z: the block CG's window SpMM in dot mode (p.Ap partials per window + fold, no k_pcg_dot pass):
# parity (windows, CG, full-size configs), then the configs[4] CG leg fused vs the separate pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05z; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_dia.py tests/test_gpu_cg.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; exit 1; }
bash tools/lab/ab_env.sh $OUT/cg 2 "bench.py --only cg_multi --no-cpu" "MSPMV_DIA_DOT=0" "MSPMV_DIA_DOT=1" || exit 1
