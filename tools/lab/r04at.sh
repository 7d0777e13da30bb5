#!/bin/bash
# r04at: L-wide SpMM tile staging in aligned pairs (pst: one 8-B column load + one 16-B value load per
# two nonzeros, as the single-RHS tile's group staging) vs tree (one 4-B + one 8-B load per nonzero),
# alternating: configs[4] CG and its SpMM, then the SpMM shapes (cant L = 16 takes the plain tile form).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04at; mkdir -p $OUT
bash tools/lab/ab_libs.sh $OUT/cg 2 tools/lab/cgmulti_probe.py tree libmspmv_pst.so || exit 1
bash tools/lab/ab_libs.sh $OUT/spmm 2 tools/lab/spmm_probe.py tree libmspmv_pst.so || exit 1
