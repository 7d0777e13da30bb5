#!/bin/bash
# r05p: offset windows (mspmv_dia.hip): parity tests, then windows vs tiles (alternating), then the
# configs[4] CG leg both ways.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05p; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dia.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -4 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; exit 1; }
bash tools/lab/ab_env.sh $OUT/ab 2 tools/lab/dia_probe.py "MSPMV_DIA=0" "MSPMV_DIA=" || exit 1
bash tools/lab/ab_env.sh $OUT/cg 1 "bench.py --only cg_multi --no-cpu" "MSPMV_DIA=0" "MSPMV_DIA=" || exit 1
