#!/bin/bash
# r06n: cant / rma10 tile stamps with the stamped kernel at the production occupancy (8 per CU); the windows
# pipelined CG fault test.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06n; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/tile_stamps.py --reps 2 > $OUT/tile_stamps.jsonl 2>$OUT/tile_stamps.err || { echo "stamps rc=$?"; tail -5 $OUT/tile_stamps.err; exit 1; }
python -c "
import json
for l in open('$OUT/tile_stamps.jsonl'):
    d=json.loads(l)
    for m in ('cold','warm'):
        c=d[m][0]; print(d['shape'], m, d['hot_kernel_us'], d['cold_kernel_us'], c['tiles'], c['max_resident'], c['span_us'], c['tile_life_us'], c['phase_median_us'], c['last_tile_entry_us'])
"
timeout -k 10 600 python -u -m pytest tests/test_gpu_faults.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
echo done
