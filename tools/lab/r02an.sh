#!/bin/bash
# Node-block SpMM compiled for the plan's tallest run (KR = 6 on 6-DOF FEM: 60 VGPRs, 8 waves/SIMD)
# vs the 8-row kernel (libmspmv_kr8.so): node-block parity tests, then SpMM times alternating.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02an; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_blocks.py tests/test_gpu_fullsize.py tests/test_gpu_cg.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in new kr8; do
    if [ $v = new ]; then lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; else lib=$PWD/tools/lab/libmspmv_kr8.so; fi
    MSPMV_LIB=$lib timeout -k 10 180 python tools/lab/spmm_probe.py > $O/s_${v}_$i.json 2> $O/s_${v}_$i.err
    rc=$?; echo "$v $i rc=$rc $(cat $O/s_${v}_$i.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
