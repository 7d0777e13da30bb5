#!/bin/bash
# r04ax: CG streaming-pass workgroups per CU after the cache policy -- tree (at most 3) vs cap2 / cap4,
# alternating, configs[4] CG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04ax; mkdir -p $OUT
bash tools/lab/ab_libs.sh $OUT/cg 3 tools/lab/cgmulti_probe.py tree libmspmv_cap2.so libmspmv_cap4.so || exit 1
