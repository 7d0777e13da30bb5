#!/bin/bash
# SpMM row-group size forced (MSPMV_SPMM_LG = 0, 1, 2: 1, 2, 4 nonzero lanes per row) vs the cost
# model, nlpkkt120 L = 8 SpMM and CG per iteration.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02ad; mkdir -p $O
for i in 1 2; do
  for v in def 1 2 3; do
    if [ $v = def ]; then unset MSPMV_SPMM_LG; else export MSPMV_SPMM_LG=$v; fi
    PROBE_SHAPE=nlpkkt timeout -k 10 180 python tools/cg_probe.py --child > $O/n_${v}_$i.json 2> $O/n_${v}_$i.err
    rc=$?; echo "lg=$v $i rc=$rc $(grep -o 'spmv_kernel_us[^}]*' $O/n_${v}_$i.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
