#!/bin/bash
# Single-RHS row-group size forced (MSPMV_SPMV_LG = 0, 1, 2, 3: 1, 2, 4, 8 lanes per row) vs the cost
# model, on the nlpkkt120-size SpMV (27-point rows) and the parabolic_fem CG (no test gate: the SpMV tests pin the default model's choices; parity of every G is covered there).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02au; mkdir -p $O
for v in def 0 1 2 3; do
  if [ $v = def ]; then unset MSPMV_SPMV_LG; else export MSPMV_SPMV_LG=$v; fi
  timeout -k 10 300 python bench.py --only cg_multi --no-cpu > $O/n_$v.json 2> $O/n_$v.err || { tail -3 $O/n_$v.err; exit 1; }
  timeout -k 10 120 python tools/cg_probe.py --child > $O/c_$v.json 2> $O/c_$v.err || exit 1
  python3 -c "import json; n=json.load(open('$O/n_$v.json')); c=json.load(open('$O/c_$v.json')); print('lg=$v', 'nlpkkt spmv', n.get('spmv_nlpkkt120_size', {}).get('kernel_ms'), 'parabolic spmv', c['spmv_kernel_us'], 'cg', c['cg_us_per_iter'])"
done
