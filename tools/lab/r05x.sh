#!/bin/bash
# r05x: offset windows after the VALU cuts of the L-wide kernel (scalar-base span addresses, no selects for
# offsets every row holds): parity, tiles vs windows at L = 1, 2, 4, 8, 16, and the configs[4] CG leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05x; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dia.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; exit 1; }
export PROBE_L="1 2 4 8 16"
bash tools/lab/ab_env.sh $OUT/ab 2 tools/lab/dia_probe.py "MSPMV_DIA=0" "MSPMV_DIA_SPMM=1" || exit 1
bash tools/lab/ab_env.sh $OUT/cg 1 "bench.py --only cg_multi --no-cpu" "MSPMV_DIA_SPMM=0" "MSPMV_DIA_SPMM=1" || exit 1
