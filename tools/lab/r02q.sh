#!/bin/bash
# k_spmm_blk gather batch (passes in flight): tree (4) vs lab 2 / 8, spmm16 leg (pwtk is the node-block case).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02q; mkdir -p $O
for i in 1 2; do
  for v in tree pb2 pb8; do
    if [ $v = tree ]; then lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; else lib=$PWD/tools/lab/libmspmv_$v.so; fi
    MSPMV_LIB=$lib timeout -k 10 300 python bench.py --only spmm16 --no-cpu > $O/s_${v}_$i.json 2>$O/s_${v}_$i.err || exit $?
    python -c "import json;d=json.load(open('$O/s_${v}_$i.json'))['pwtk'];print('$v', d['hot_kernel_ms'], d['cold_kernel_ms'], d['frac'])"
  done
done
