#!/bin/bash
# SpMM row-group remainder in one predicated batch (instead of single-gather round trips): parity
# tests, then SpMM kernel times and the nlpkkt120 L = 8 CG per iteration, base vs in-tree.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02ac; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_spmv.py tests/test_gpu_blocks.py tests/test_gpu_fullsize.py tests/test_gpu_cg.py tests/test_spai.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/lab/ab_spmm.sh $O 2 || exit 1
for i in 1 2; do
  for v in base new; do
    if [ $v = base ]; then lib=$PWD/tools/lab/libmspmv_base.so; else lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; fi
    MSPMV_LIB=$lib PROBE_SHAPE=nlpkkt timeout -k 10 180 python tools/cg_probe.py --child > $O/n_${v}_$i.json 2> $O/n_${v}_$i.err
    rc=$?; echo "nlpkkt $v $i rc=$rc $(grep -o 'spmv_kernel_us[^}]*' $O/n_${v}_$i.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
