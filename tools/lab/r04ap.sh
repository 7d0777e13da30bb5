#!/bin/bash
# r04ap: single-RHS SpMV row stores nontemporal (nty: plain SpMV forms only; y is not re-read by the
# launch) vs tree, alternating, on the bench shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04ap; mkdir -p $OUT
PROBE_SHAPES="pwtk pwtk_perturbed nlpkkt scatter cant powerlaw" bash tools/lab/ab_libs.sh $OUT/spmv 2 tools/lab/spmv_probe.py tree libmspmv_nty.so || exit 1
