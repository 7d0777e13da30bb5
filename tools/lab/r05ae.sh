#!/bin/bash
# r05ae: L-wide offset windows with LDS-DMA span staging (MSPMV_DIA_DMA=1): parity under it, then alternating
# timings at L = 2, 4, 8, 16 on the nlpkkt120 size and the configs[4] CG leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05ae; mkdir -p $OUT
MSPMV_DIA_DMA=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_dia.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; exit 1; }
export PROBE_L="2 4 8 16" PROBE_ONLY="nlpkkt"
bash tools/lab/ab_env.sh $OUT/ab 2 tools/lab/dia_probe.py "MSPMV_DIA_DMA=0" "MSPMV_DIA_DMA=1" || exit 1
bash tools/lab/ab_env.sh $OUT/cg 2 "bench.py --only cg_multi --no-cpu" "MSPMV_DIA_DMA=0" "MSPMV_DIA_DMA=1" || exit 1
