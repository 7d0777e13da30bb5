#!/bin/bash
# A/B: k_spmv_blk (one tile per workgroup) vs k_spmv_runs (persistent, wave-pipelined) on the
# headline pwtk-shaped SpMV, after the node-block parity tests with the new kernel forced on.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02l; mkdir -p $O
MSPMV_SPMV_RUNS=1 timeout -k 10 300 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 \
    tests/test_gpu_blocks.py > $O/pytest_runs.log 2>&1 || { tail -30 $O/pytest_runs.log; exit 1; }
tail -2 $O/pytest_runs.log
for i in 1 2 3; do
  for r in 0 1; do
    MSPMV_SPMV_RUNS=$r timeout -k 10 300 python bench.py --no-cpu --no-cg --no-extras --steps 400 > $O/b_${r}_$i.json 2>$O/b_${r}_$i.err || exit $?
    python -c "import json;d=json.load(open('$O/b_${r}_$i.json'));r=d['roofline'];print('runs=$r', d['value'], r['kernel'], r['kernel_ms'], r['frac'])"
  done
done
