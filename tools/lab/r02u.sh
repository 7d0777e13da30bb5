#!/bin/bash
# Tile slots per CU for the single-RHS CG plan: default (attribute-based, MSPMV_DEBUG_SLOTS prints the
# runtime query too) vs forced 0 (no stretch), 7, 8; parabolic_fem-shaped CG per iteration, 2 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02u; mkdir -p $O
for i in 1 2; do
  for v in def 0 7 8; do
    if [ $v = def ]; then env=""; else env="MSPMV_TILE_SLOTS_PER_CU=$v"; fi
    env MSPMV_DEBUG_SLOTS=1 $env timeout -k 10 120 python tools/cg_probe.py --child > $O/cg_${v}_$i.json 2> $O/cg_${v}_$i.err
    rc=$?; echo "$v $i rc=$rc $(cat $O/cg_${v}_$i.json) $(grep slots $O/cg_${v}_$i.err)"; [ $rc -eq 0 ] || exit $rc
  done
done
