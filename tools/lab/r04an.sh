#!/bin/bash
# r04an: tree (r04al + r04am: x, Ap, p-in-p.Ap, r-in-p-update loaded nontemporal) vs ntu (r loaded
# nontemporal in the r update too), alternating, configs[4] CG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04an; mkdir -p $OUT
bash tools/lab/ab_libs.sh $OUT/cg 3 tools/lab/cgmulti_probe.py tree libmspmv_ntu.so || exit 1
