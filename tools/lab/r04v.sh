#!/bin/bash
# r04v: where the column-slab SpMV's time goes -- tree vs noent (no run sums into yacc) vs noprod
# (products without the LDS x gather) vs nox (no slab loads after the first), forced on, scattered
# band, alternating (timing only: the variants compute wrong rows).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04v; mkdir -p $OUT
export PROBE_SHAPES="scatter" MSPMV_SPMV_SLAB=1
bash tools/lab/ab_libs.sh $OUT/spmv 2 tools/lab/spmv_probe.py tree libmspmv_noent.so libmspmv_noprod.so libmspmv_nox.so || exit 1
