#!/bin/bash
# Sharded CG batch graph: dist GPU tests (graph == eager bit for bit), then per-iteration time
# eager vs graph at world 1 (parabolic_fem L = 1, nlpkkt120 L = 8; whole-local and split iteration).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02w; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_dist.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|SKIP|ERROR|passed|failed" $O/tests.log | tail -14; [ $rc -eq 0 ] || exit $rc
for cfg in "parabolic 1" "nlpkkt 8"; do
  for split in 0 1; do
    for g in 0 1; do
      MSPMV_DIST_GRAPH=$g MSPMV_DIST_FORCE_SPLIT=$split timeout -k 10 180 python tools/lab/dist_graph_probe.py $cfg > $O/p.json 2> $O/p.err
      rc=$?; echo "rc=$rc $(cat $O/p.json)"; [ $rc -eq 0 ] || { tail -5 $O/p.err; exit $rc; }
    done
  done
done
