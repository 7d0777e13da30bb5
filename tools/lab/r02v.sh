#!/bin/bash
# Deferred x update in both CG forms: CG parity tests, then A/B (tools/lab/libmspmv_base.so vs in-tree)
# of the CG per-iteration time on the parabolic_fem (L = 1) and nlpkkt120 (L = 8) shapes.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02v; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_cg.py tests/test_gpu_blocks.py tests/test_gpu_dist.py tests/test_spai.py tests/test_ic0.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for shape in parabolic nlpkkt; do
  for i in 1 2; do
    for v in base new; do
      if [ $v = base ]; then lib=$PWD/tools/lab/libmspmv_base.so; else lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; fi
      PROBE_SHAPE=$shape MSPMV_LIB=$lib timeout -k 10 180 python tools/cg_probe.py --child > $O/${shape}_${v}_$i.json 2> $O/${shape}_${v}_$i.err
      rc=$?; echo "$shape $v $i rc=$rc $(cat $O/${shape}_${v}_$i.json)"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
