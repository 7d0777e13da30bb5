#!/bin/bash
# r04aq: tree vs ntq (Ap also loaded nontemporal in the p.Ap pass), alternating, configs[4] CG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04aq; mkdir -p $OUT
bash tools/lab/ab_libs.sh $OUT/cg 3 tools/lab/cgmulti_probe.py tree libmspmv_ntq.so || exit 1
