#!/bin/bash
# r04l: split rows closed in the tile kernels -- A/B of head (k_fixup launch), tree (last-arriver
# tickets, heads redirected to a slot, FIX=false kernels for plans without split rows), sc1row (the
# first attempt: every tile's row 0 stored with agent scope) on the SpMV shapes; configs[4] with
# head / tree / nty (r04j's nontemporal Y stores); then the split-row tests and the GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04l; mkdir -p $OUT
export PROBE_SHAPES="nlpkkt powerlaw cant pwtk"
timeout -k 10 300 python -m pytest tests/test_gpu_split_rows.py -m gpu -q -p no:cacheprovider -rf > $OUT/split_tests.log 2>&1
rc=$?; echo "split tests rc=$rc"; tail -5 $OUT/split_tests.log; [ $rc -le 1 ] || exit $rc
bash tools/lab/ab_libs.sh $OUT/spmv 2 tools/lab/spmv_probe.py tree libmspmv_head.so libmspmv_sc1row.so || exit 1
for v in tree libmspmv_head.so libmspmv_nty.so; do
  if [ $v = tree ]; then lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; else lib=$PWD/tools/lab/$v; fi
  MSPMV_LIB=$lib timeout -k 10 200 python3 tools/lab/cgmulti_probe.py > $OUT/cg_$v.txt 2>$OUT/cg_$v.err || { echo "$v rc=$?"; tail -3 $OUT/cg_$v.err; exit 1; }
  echo "cg $v $(cat $OUT/cg_$v.txt)"
done
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -rf > $OUT/pytest_gpu.log 2>&1
echo "gpu tests rc=$?"; tail -8 $OUT/pytest_gpu.log
