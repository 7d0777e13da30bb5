#!/bin/bash
# Node-block SpMM with LDS value broadcast (now default): passes in flight per batch, in-tree
# (4 at L = 16, 2 below) vs 2 / 4 / 8 everywhere; node-block tests on the in-tree build first.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02ah; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_blocks.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in new pb2 pb4 pb8; do
    if [ $v = new ]; then lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; else lib=$PWD/tools/lab/libmspmv_$v.so; fi
    MSPMV_LIB=$lib timeout -k 10 180 python tools/lab/spmm_probe.py > $O/s_${v}_$i.json 2> $O/s_${v}_$i.err
    rc=$?; echo "$v $i rc=$rc $(cat $O/s_${v}_$i.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
