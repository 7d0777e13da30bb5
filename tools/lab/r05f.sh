#!/bin/bash
# r05f: warp-specialized column-slab SpMM (stream waves 4 chunks ahead in registers, panel waves by
# LDS-DMA one segment ahead): parity tests, then tiles vs slab configurations.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05f; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_slab_mm.py -x -v --timeout 120 --timeout-method thread -k "not default_choice" > $OUT/pytest.log 2>&1
rc=$?
tail -4 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; exit 1; }
bash tools/lab/ab_env.sh $OUT/ab 1 tools/lab/slabmm_probe.py "MSPMV_SPMM_SLAB=0" "MSPMV_SPMM_SLAB=1" \
  "MSPMV_SPMM_SLAB=1 MSPMV_SPMM_SLAB_CFG=1" "MSPMV_SPMM_SLAB=1 MSPMV_SPMM_SLAB_CFG=3" || exit 1
