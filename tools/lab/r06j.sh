#!/bin/bash
# r06j: what bounds the L = 8 window SpMM: ablations (MSPMV_DIA_EXACT bits: 2 = every window's values from
# window 0's panels (L2-resident), 4 = every span from X rows 0..66 (L1/L2-resident)); results wrong, timing only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06j; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for ab in 0 2 4 6; do
    for L in 8 1; do
      MSPMV_DIA_EXACT=$ab PROBE_L=$L timeout -k 10 300 python tools/lab/spmm8_probe.py > $OUT/p_${ab}_${L}_$i.json 2>$OUT/p_${ab}_${L}_$i.err || { echo "probe rc=$?"; tail -3 $OUT/p_${ab}_${L}_$i.err; exit 1; }
      echo "ab=$ab $(cat $OUT/p_${ab}_${L}_$i.json)"
    done
  done
done
echo done
