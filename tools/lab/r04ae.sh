#!/bin/bash
# r04ae: configs[4]'s streaming passes -- tree (<= 2,048 blocks, ~4 pairs per thread) vs vb4k
# (<= 4,096, ~2) vs vb1k (<= 1,024, ~8), alternating; rerun as r04af: tree, vb1k, vb768 (<= 768), vb512 (<= 512).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/${TAG:-r04ae}; mkdir -p $OUT
bash tools/lab/ab_libs.sh $OUT/cg 2 tools/lab/cgmulti_probe.py tree libmspmv_vb1k.so libmspmv_vb768.so libmspmv_vb512.so || exit 1
