#!/bin/bash
# r05ab: the L = 1 window kernel with unguarded full batches and a select-free path for full windows,
# against the previous build (tools/lab/libmspmv_base.so): parity, then alternating timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05ab; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dia.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; exit 1; }
export PROBE_L="1"
bash tools/lab/ab_env.sh $OUT/ab 3 tools/lab/dia_probe.py "MSPMV_LIB=tools/lab/libmspmv_base.so" "MSPMV_LIB=" || exit 1
