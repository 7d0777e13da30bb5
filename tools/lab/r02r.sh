#!/bin/bash
# k_spmm_blk with fused multiply-adds and the row-length test hoisted (lab build "fma") vs tree:
# node-block parity tests on the lab build, then the spmm16 leg A/B.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02t; mkdir -p $O
for L in tree fma; do if [ $L = tree ]; then LIBP=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; else LIBP=$PWD/tools/lab/libmspmv_fma.so; fi; MSPMV_LIB=$LIBP timeout -k 10 300 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 \
    tests/test_gpu_blocks.py tests/test_gpu_spmv.py > $O/pytest_$L.log 2>&1 || { tail -30 $O/pytest_$L.log; exit 1; }; tail -1 $O/pytest_$L.log; done
for i in 1 2; do
  for v in tree fma; do
    if [ $v = tree ]; then lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; else lib=$PWD/tools/lab/libmspmv_$v.so; fi
    MSPMV_LIB=$lib timeout -k 10 300 python bench.py --only spmm16 --no-cpu > $O/s_${v}_$i.json 2>$O/s_${v}_$i.err || exit $?
    python -c "import json;d=json.load(open('$O/s_${v}_$i.json'))['pwtk'];print('$v', d['hot_kernel_ms'], d['cold_kernel_ms'], d['frac'])"
  done
done
