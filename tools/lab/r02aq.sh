#!/bin/bash
# SpMM tile kernels with the waves-per-EU cap at 8 (libmspmv_w8.so: L = 16 at 63 VGPRs, 2 spilled)
# vs without (in-tree): node-block parity tests on the variant, then SpMM times alternating.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02aq; mkdir -p $O
MSPMV_LIB=$PWD/tools/lab/libmspmv_w8.so timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_spmv.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in new w8; do
    if [ $v = new ]; then lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; else lib=$PWD/tools/lab/libmspmv_w8.so; fi
    MSPMV_LIB=$lib timeout -k 10 180 python tools/lab/spmm_probe.py > $O/s_${v}_$i.json 2> $O/s_${v}_$i.err
    rc=$?; echo "$v $i rc=$rc $(cat $O/s_${v}_$i.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
