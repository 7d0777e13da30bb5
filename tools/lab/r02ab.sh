#!/bin/bash
# Tail split of large single-RHS plans (half-size tiles closing every XCD's tile range) vs uniform
# tiles (MSPMV_SPMV_TAIL=0): SpMV parity tests, then the bench headline + nlpkkt120-size SpMV, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_spmv.py tests/test_gpu_blocks.py tests/test_gpu_fullsize.py tests/test_gpu_cg.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in 1 0; do
    MSPMV_DEBUG_SLOTS=1 MSPMV_SPMV_TAIL=$v timeout -k 10 300 python bench.py --no-cpu --no-cg > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 $O/b_${v}_$i.err; exit $rc; }
    python3 -c "
import json,sys; d=json.load(open('$O/b_${v}_$i.json'))
print("tail=$v", d["value"], d["roofline"]["frac"], d["roofline"]["kernel_ms"], "scatter", d["scatter_band_stress"]["kernel_ms"])"
  done
done
grep -h "slots\|tail split" $O/b_1_1.err | head -5
