#!/bin/bash
# r04ai: L = 8 SpMM tile depth -- tree (16 items per lane group: ~37 stencil rows per 1,024-item tile)
# vs k20 / k24 / k28 / k32 (1,280 / 1,536 / 1,792 / 2,048 items), alternating: the configs[4] CG and
# its SpMM, then the SpMM bench shapes (pwtk L = 2..16, cant and nlpkkt).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04ai; mkdir -p $OUT
bash tools/lab/ab_libs.sh $OUT/cg 2 tools/lab/cgmulti_probe.py tree libmspmv_k20.so libmspmv_k24.so libmspmv_k28.so libmspmv_k32.so || exit 1
bash tools/lab/ab_libs.sh $OUT/spmm 2 tools/lab/spmm_probe.py tree libmspmv_k24.so libmspmv_k28.so libmspmv_k32.so || exit 1
