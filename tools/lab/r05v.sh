#!/bin/bash
# r05v: offset windows with paired value panels (16-B loads at L = 1) and the LDS-run L-wide kernel:
# parity, then tiles vs windows on the probe shapes and on the configs[4] CG leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05v; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dia.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; exit 1; }
bash tools/lab/ab_env.sh $OUT/ab 2 tools/lab/dia_probe.py "MSPMV_DIA=0" "MSPMV_DIA_SPMM=1" || exit 1
bash tools/lab/ab_env.sh $OUT/cg 1 "bench.py --only cg_multi --no-cpu" "MSPMV_DIA_SPMM=0" "MSPMV_DIA_SPMM=1" || exit 1
