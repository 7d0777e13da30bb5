#!/bin/bash
# r04n: configs[4] and the L-wide SpMM -- tree vs nty (nontemporal Y stores in k_spmm_tile) vs nog
# (panel gathers folded onto 1,024 L1-resident rows: what the gathers cost; SpMM only -- its CG
# cannot converge), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04n; mkdir -p $OUT
bash tools/lab/ab_libs.sh $OUT/spmm 2 tools/lab/spmm_probe.py tree libmspmv_nty.so libmspmv_nog.so || exit 1
bash tools/lab/ab_libs.sh $OUT/cg 1 tools/lab/cgmulti_probe.py tree libmspmv_nty.so || exit 1
