#!/bin/bash
# r04d: A/B of the node-block SpMV kernel: tree vs no fallback path vs no register caps vs r03; noshift on nlpkkt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04d; mkdir -p $OUT
L=$PWD/tools/lab
for rep in 1 2; do
  for v in tree nofb noattr r03; do
    if [ $v = tree ]; then lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; else lib=$L/libmspmv_$v.so; fi
    MSPMV_LIB=$lib timeout -k 10 200 python3 tools/lab/spmv_probe.py pwtk > $OUT/${v}_$rep.txt 2>$OUT/${v}_$rep.err || { echo "$v rc=$?"; tail -3 $OUT/${v}_$rep.err; exit 1; }
    echo "$v $rep $(cat $OUT/${v}_$rep.txt)"
  done
  for v in tree noshift; do
    if [ $v = tree ]; then lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; else lib=$L/libmspmv_$v.so; fi
    MSPMV_LIB=$lib timeout -k 10 200 python3 tools/lab/spmv_probe.py nlpkkt pwtk_perturbed > $OUT/${v}_nl_$rep.txt 2>$OUT/${v}_nl_$rep.err || { echo "$v rc=$?"; tail -3 $OUT/${v}_nl_$rep.err; exit 1; }
    echo "$v $rep $(cat $OUT/${v}_nl_$rep.txt)"
  done
done
