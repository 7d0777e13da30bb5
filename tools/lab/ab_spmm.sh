#!/bin/bash
# A/B of the SpMM kernels: tools/lab/libmspmv_base.so vs the in-tree library, alternating.
#   usage: tools/lab/ab_spmm.sh OUTDIR [reps]
cd "$(dirname "$0")/../.."
OUT=$1; REPS=${2:-2}
mkdir -p "$OUT"
for i in $(seq 1 "$REPS"); do
  for v in base new; do
    if [ $v = base ]; then lib=$PWD/tools/lab/libmspmv_base.so; else lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; fi
    MSPMV_LIB=$lib timeout -k 10 180 python tools/lab/spmm_probe.py > "$OUT/spmm_${v}_$i.json" 2>"$OUT/spmm_${v}_$i.err" || { echo "$v rc=$?"; tail -3 "$OUT/spmm_${v}_$i.err"; exit 1; }
    echo "$v $i $(cat "$OUT/spmm_${v}_$i.json")"
  done
done
