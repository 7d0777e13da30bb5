#!/bin/bash
# r04az: the CG's SpMM stores Ap with plain (temporal) stores (yt; the p.Ap pass reads it next) vs tree
# (nontemporal, as every SpMM), alternating, configs[4] CG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04az; mkdir -p $OUT
bash tools/lab/ab_libs.sh $OUT/cg 3 tools/lab/cgmulti_probe.py tree libmspmv_yt.so || exit 1
