#!/bin/bash
# r06cc: one-shot HBM read ceiling at the small matrices' sizes (cant 49.3 MB, rma10 29.4 MB; copies rotating through
# > 600 MB so every launch reads from HBM), kernel durations from the trace (per-launch events add ~4.7 us).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06cc; mkdir -p $OUT
export TMPDIR=/tmp
for sz in 49337620 29424716 142651548; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$sz -o rc -- ./tools/read_ceiling $sz > $OUT/rc_$sz.txt 2>$OUT/rc_$sz.err || { echo "rc=$?"; tail -3 $OUT/rc_$sz.err; exit 1; }
  echo "== $sz"; grep -v "^==" $OUT/rc_$sz.txt | head -20
done
echo done
