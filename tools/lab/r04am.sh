#!/bin/bash
# r04am: on top of r04al's nontemporal x (p update) and Ap (r update): ntp (p loaded nontemporal in
# the p.Ap pass: next read two passes on) vs ntr (r loaded nontemporal in the p update) vs ntpr,
# alternating, configs[4] CG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04am; mkdir -p $OUT
bash tools/lab/ab_libs.sh $OUT/cg 3 tools/lab/cgmulti_probe.py tree libmspmv_ntp.so libmspmv_ntr.so libmspmv_ntpr.so || exit 1
