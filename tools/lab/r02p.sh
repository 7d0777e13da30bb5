#!/bin/bash
# CG single (parabolic_fem shape): tile depth (MSPMV_SPMV_IPT) A/B on the tree build.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02p; mkdir -p $O
for i in 1 2; do
  for ipt in 8 4 6 7; do
    MSPMV_SPMV_IPT=$ipt timeout -k 10 300 python bench.py --only cg_single --no-cpu > $O/cg_${ipt}_$i.json 2>$O/cg_${ipt}_$i.err || exit $?
    python -c "import json;d=json.load(open('$O/cg_${ipt}_$i.json'));print('ipt=$ipt', d['iterations'], d['us_per_iter'], d['roofline_frac'])"
  done
done
