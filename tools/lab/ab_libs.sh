#!/bin/bash
# A/B/C of library variants on one probe, alternating, each run in its own process.
#   usage: tools/lab/ab_libs.sh OUTDIR REPS PROBE.py lib1.so [lib2.so ...]   (in-tree lib: "tree")
cd "$(dirname "$0")/../.."
OUT=$1; REPS=$2; PROBE=$3; shift 3
mkdir -p "$OUT"
for i in $(seq 1 "$REPS"); do
  for v in "$@"; do
    if [ "$v" = tree ]; then lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; else lib=$PWD/tools/lab/$v; fi
    n=$(basename "$v" .so)
    MSPMV_LIB=$lib timeout -k 10 180 python "$PROBE" > "$OUT/${n}_$i.json" 2>"$OUT/${n}_$i.err" || { echo "$v rc=$?"; tail -3 "$OUT/${n}_$i.err"; exit 1; }
    echo "$n $i $(cat "$OUT/${n}_$i.json")"
  done
done
