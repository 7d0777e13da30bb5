#!/bin/bash
# A/B of the single-RHS CG: tools/lab/libmspmv_base.so (saved before a change) vs the in-tree
# library, alternating, each probe in its own process.   usage: tools/lab/ab_cg.sh OUTDIR [reps]
cd "$(dirname "$0")/../.."
OUT=$1; REPS=${2:-2}
mkdir -p "$OUT"
for i in $(seq 1 "$REPS"); do
  for v in base new; do
    if [ $v = base ]; then lib=$PWD/tools/lab/libmspmv_base.so; else lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; fi
    MSPMV_LIB=$lib timeout -k 10 120 python tools/cg_probe.py --child > "$OUT/cg_${v}_$i.json" 2>"$OUT/cg_${v}_$i.err" || { echo "$v rc=$?"; exit 1; }
    echo "$v $i $(grep '^{' "$OUT/cg_${v}_$i.json")"
  done
done
