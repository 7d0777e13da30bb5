#!/bin/bash
# r04ad: the L = 16 SpMM's row groups on cant -- tree vs b16 (16 panel-row gathers in flight per
# lane instead of 8) vs lg2x (row groups forced to 4 nonzero lanes), alternating; the spmm16 bench
# leg (cold, with the kernel name) on the tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04ad; mkdir -p $OUT
bash tools/lab/ab_libs.sh $OUT/spmm 2 tools/lab/spmm_probe.py tree libmspmv_b16.so libmspmv_lg2x.so || exit 1
timeout -k 10 400 python bench.py --only spmm16 > $OUT/spmm16.json 2>$OUT/spmm16.err; echo "leg rc=$?"; tail -1 $OUT/spmm16.json
