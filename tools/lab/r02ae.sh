#!/bin/bash
# Pipelined CG: update blocks 1024 (default) vs 512 / 256 (MSPMV_CG1_BLOCKS), parabolic_fem shape.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02ae; mkdir -p $O
for i in 1 2; do
  for v in 1024 512 256; do
    MSPMV_CG1_BLOCKS=$v timeout -k 10 180 python tools/cg_probe.py --child > $O/c_${v}_$i.json 2> $O/c_${v}_$i.err
    rc=$?; echo "blocks=$v $i rc=$rc $(grep -o 'cg_us_per_iter[^}]*' $O/c_${v}_$i.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
