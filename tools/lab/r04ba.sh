#!/bin/bash
# r04ba: the split CG's p.Ap from the SpMM's dot mode (MSPMV_CG_DOT=fused) vs its own pass (default),
# alternating, configs[4] CG, after round 4's tile depth, pair staging and cache policy.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04ba; mkdir -p $OUT
for i in 1 2 3; do
  for mode in pass fused; do
    if [ $mode = fused ]; then export MSPMV_CG_DOT=fused; else unset MSPMV_CG_DOT; fi
    timeout -k 10 180 python tools/lab/cgmulti_probe.py > $OUT/${mode}_$i.json 2> $OUT/${mode}_$i.err || { echo "$mode rc=$?"; tail -3 $OUT/${mode}_$i.err; exit 1; }
    echo "$mode $i $(cat $OUT/${mode}_$i.json)"
  done
done
