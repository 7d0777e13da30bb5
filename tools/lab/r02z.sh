#!/bin/bash
# (1) GPU tests of the tile-kernel changes (no-block CG variant, multi-generation stretch);
# (2) pipelined CG at IPT 8 vs 4 (parabolic_fem shape; IPT 4's no-block CG kernel: 60 VGPRs);
# (3) k_spmm_blk variants (PB 2, waves 6/7) vs the in-tree library.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02z; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_cg.py tests/test_gpu_spmv.py tests/test_gpu_blocks.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  MSPMV_DEBUG_SLOTS=1 PROBE_VARIANTS="8:48,4:48" timeout -k 10 400 python tools/cg_probe.py > $O/cg_$i.txt 2>&1
  rc=$?; echo "cg probe $i rc=$rc"; cat $O/cg_$i.txt | grep -v "^mspmv"; [ $rc -eq 0 ] || exit $rc
done
for v in new pb2 w6pb2 w7pb2; do
  if [ $v = new ]; then lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; else lib=$PWD/tools/lab/libmspmv_$v.so; fi
  [ -f $lib ] || continue
  MSPMV_LIB=$lib timeout -k 10 180 python tools/lab/spmm_probe.py > $O/spmm_$v.json 2> $O/spmm_$v.err
  rc=$?; echo "spmm $v rc=$rc $(cat $O/spmm_$v.json)"; [ $rc -eq 0 ] || exit $rc
done
