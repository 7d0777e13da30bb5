#!/bin/bash
# r04o: what bounds the L-wide SpMM tile kernel -- tree vs g64 (panel gathers folded onto 64
# L1-resident rows) vs g0 (no gather: the value is formed from the column id), SpMM only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04o; mkdir -p $OUT
bash tools/lab/ab_libs.sh $OUT/spmm 2 tools/lab/spmm_probe.py tree libmspmv_g64.so libmspmv_g0.so libmspmv_nog.so || exit 1
