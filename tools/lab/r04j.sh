#!/bin/bash
# r04j: configs[4] A/B: tree vs nty (nontemporal Y stores in the L-wide SpMM)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04j; mkdir -p $OUT
for rep in 1 2; do
  for v in tree nty; do
    if [ $v = tree ]; then lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; else lib=$PWD/tools/lab/libmspmv_$v.so; fi
    MSPMV_LIB=$lib timeout -k 10 200 python3 tools/lab/cgmulti_probe.py > $OUT/${v}_$rep.txt 2>$OUT/${v}_$rep.err || { echo "$v rc=$?"; tail -3 $OUT/${v}_$rep.err; exit 1; }
    echo "$v $rep $(cat $OUT/${v}_$rep.txt)"
  done
done
