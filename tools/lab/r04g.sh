#!/bin/bash
# r04g: A/B of the pair staging's x loads: tree (two 8-B gathers per pair) vs xadj (one 16-B load per adjacent pair)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04g; mkdir -p $OUT
for rep in 1 2; do
  for v in tree xadj; do
    if [ $v = tree ]; then lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; else lib=$PWD/tools/lab/libmspmv_$v.so; fi
    MSPMV_LIB=$lib timeout -k 10 200 python3 tools/lab/spmv_probe.py nlpkkt cant scatter > $OUT/${v}_$rep.txt 2>$OUT/${v}_$rep.err || { echo "$v rc=$?"; tail -3 $OUT/${v}_$rep.err; exit 1; }
    python3 -c "
import json,sys
for l in open('$OUT/${v}_$rep.txt'): d=json.loads(l); print('$v', $rep, d['shape'], d['kernel'], d['kernel_us'], d['frac'])"
  done
done
