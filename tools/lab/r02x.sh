#!/bin/bash
# Split CG p.Ap: separate pass after the plain SpMM (default) vs the SpMM's dot mode (MSPMV_CG_DOT=fused).
# CG parity tests on the default, then per-iteration A/B on the nlpkkt120 L = 8 shape (+ L = 1 split).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02x; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_cg.py tests/test_gpu_blocks.py tests/test_spai.py tests/test_ic0.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in pass fused; do
    MSPMV_CG_DOT=$v PROBE_SHAPE=nlpkkt timeout -k 10 180 python tools/cg_probe.py --child > $O/n_${v}_$i.json 2> $O/n_${v}_$i.err
    rc=$?; echo "nlpkkt $v $i rc=$rc $(cat $O/n_${v}_$i.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
