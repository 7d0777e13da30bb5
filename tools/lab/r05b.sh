#!/bin/bash
# r05b: the column-slab SpMM after static prefetch counts (no vmcnt(0) drain, panel registers out of scratch)
# cant L = 16 and the nlpkkt120-size L = 8 SpMM / CG, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05b; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_slab_mm.py -x -v -k "not default_choice" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -15 $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
bash tools/lab/ab_env.sh $OUT/ab 2 tools/lab/slabmm_probe.py "MSPMV_SPMM_SLAB=0" "MSPMV_SPMM_SLAB=1 MSPMV_SPMM_SLAB_CFG=0" \
  "MSPMV_SPMM_SLAB=1 MSPMV_SPMM_SLAB_CFG=1" "MSPMV_SPMM_SLAB=1 MSPMV_SPMM_SLAB_CFG=3" || exit 1
