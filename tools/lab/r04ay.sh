#!/bin/bash
# r04ay: single-RHS tile depth on the 27-point stencil -- tree (8 items per thread: 2,048-item tiles,
# ~73 rows on 128 two-lane row groups) vs ipt7 (1,792 items: ~64 rows, one round of 64 four-lane
# groups) vs ipt10, alternating, nlpkkt120 size and pwtk.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04ay; mkdir -p $OUT
PROBE_SHAPES="nlpkkt pwtk" bash tools/lab/ab_libs.sh $OUT/spmv 2 tools/lab/spmv_probe.py tree libmspmv_ipt7.so libmspmv_ipt10.so || exit 1
