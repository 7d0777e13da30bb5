#!/bin/bash
# r05g: LAB stamped build of the column-slab SpMM: per-chunk phase lengths (shader cycles)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05g; mkdir -p $OUT
timeout -k 10 300 python tools/lab/slabmm_stamps.py $OUT > $OUT/stamps.txt 2>&1; rc=$?
cat $OUT/stamps.txt; exit $rc
