#!/bin/bash
# r04bb: L = 8 tile depth re-check after the pair staging -- tree (24 items per lane group) vs q20 / q28,
# alternating, configs[4] CG and its SpMM.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04bb; mkdir -p $OUT
bash tools/lab/ab_libs.sh $OUT/cg 3 tools/lab/cgmulti_probe.py tree libmspmv_q20.so libmspmv_q28.so || exit 1
