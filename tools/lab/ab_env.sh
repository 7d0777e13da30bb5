#!/bin/bash
# A/B/C of environment variants of the in-tree library on one probe, alternating, each run in its own
# process.   usage: tools/lab/ab_env.sh OUTDIR REPS "PROBE.py [args]" "VAR=V ..." ["VAR=V ..." ...]
cd "$(dirname "$0")/../.."
OUT=$1; REPS=$2; PROBE=$3; shift 3
mkdir -p "$OUT"
for i in $(seq 1 "$REPS"); do
  k=0
  for v in "$@"; do
    k=$((k + 1))
    env $v timeout -k 10 300 python $PROBE > "$OUT/v${k}_$i.json" 2>"$OUT/v${k}_$i.err" || { echo "[$v] rc=$?"; tail -5 "$OUT/v${k}_$i.err"; exit 1; }
    echo "v$k $i $(cat "$OUT/v${k}_$i.json")"
  done
done
