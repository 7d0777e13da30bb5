#!/bin/bash
# r05ad: counter passes of the current window kernels (L = 1 and 8) and the tiles on the nlpkkt120 size.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05ad; mkdir -p $OUT
timeout -k 10 700 bash tools/pmc_passes.sh $OUT/ctr "k_spmm_dia|k_spmm_tile|k_spmv_tile" -- python3 tools/lab/dia_ctr_probe.py || exit 1
python3 tools/counter_summary.py $OUT/ctr --title "r05ad: offset windows (after the VALU cuts and L = 1 batches) vs merge tiles, nlpkkt120 size" > $OUT/counters.md
