#!/bin/bash
# r04as: L = 8 row-group gather batches -- tree (8 panel-row gathers in flight per lane: a 27-nonzero
# stencil row takes 8 + 8 + 8 + a clamped 4) vs nb9 (9 + 9 + 9) / nb12 (12 + 12 + 4) / nb16
# (16 + 8 + 4); occupancy is set by LDS (5 workgroups per CU), so up to 102 VGPRs are free.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04as; mkdir -p $OUT
bash tools/lab/ab_libs.sh $OUT/cg 2 tools/lab/cgmulti_probe.py tree libmspmv_nb9.so libmspmv_nb12.so libmspmv_nb16.so || exit 1
