#!/bin/bash
# Headline SpMV with the matrix stream's nontemporal hint forced off / on (MSPMV_SPMV_NT; auto = on
# above 128 MiB, so on for the pwtk shape), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02aw; mkdir -p $O
for i in 1 2 3; do
  for v in 1 0; do
    MSPMV_SPMV_NT=$v timeout -k 10 300 python bench.py --no-cpu --no-cg --no-extras > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit 1
    python3 -c "import json; d=json.load(open('$O/b_${v}_$i.json')); print('nt=$v', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['roofline']['kernel'])"
  done
done
