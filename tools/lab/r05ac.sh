#!/bin/bash
# r05ac: interleaved window order (MSPMV_DIA_ORDER=1: three streams one plane apart inside each XCD's
# range): parity under it, then alternating timings at L = 1 and 8 and the configs[4] CG leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05ac; mkdir -p $OUT
MSPMV_DIA_ORDER=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_dia.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; exit 1; }
export PROBE_L="1 8" PROBE_ONLY="nlpkkt"
bash tools/lab/ab_env.sh $OUT/ab 3 tools/lab/dia_probe.py "MSPMV_DIA_ORDER=0" "MSPMV_DIA_ORDER=1" || exit 1
bash tools/lab/ab_env.sh $OUT/cg 2 "bench.py --only cg_multi --no-cpu" "MSPMV_DIA_ORDER=0" "MSPMV_DIA_ORDER=1" || exit 1
