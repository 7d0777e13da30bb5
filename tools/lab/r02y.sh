#!/bin/bash
# Split CG sweep direction: alternate (MSPMV_CG_REV=1, default) vs all forward (0), nlpkkt120 L = 8,
# after the CG parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02y; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_cg.py tests/test_gpu_blocks.py tests/test_gpu_dist.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in 1 0; do
    MSPMV_CG_REV=$v PROBE_SHAPE=nlpkkt timeout -k 10 180 python tools/cg_probe.py --child > $O/n_${v}_$i.json 2> $O/n_${v}_$i.err
    rc=$?; echo "nlpkkt rev=$v $i rc=$rc $(grep -o 'cg_us_per_iter[^}]*' $O/n_${v}_$i.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
