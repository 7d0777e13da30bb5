#!/bin/bash
# r04al: nontemporal accesses in the split CG's streaming passes -- tree vs ntx (x loaded and stored
# nontemporal in the p update: x is touched once per iteration) vs nta (Ap loaded nontemporal in the
# r update: its last use) vs ntxa (both), alternating, configs[4] CG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04al; mkdir -p $OUT
bash tools/lab/ab_libs.sh $OUT/cg 3 tools/lab/cgmulti_probe.py tree libmspmv_ntx.so libmspmv_nta.so libmspmv_ntxa.so || exit 1
