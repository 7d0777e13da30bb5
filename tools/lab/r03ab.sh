#!/bin/bash
# r03ab: carry fix-up as one wave per run of a row's carries (was: one thread looping over them, 85 us
# for the skewed variant's dense row) and the fix-up inside the timed SpMV -- parity, then the shapes leg
# under a kernel trace
cd "$(dirname "$0")/../.."
OUT=$PWD/gpurun_out/r03ab; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_spmv.py tests/test_gpu_cg.py tests/test_gpu_dist.py tests/test_spai.py > $OUT/tests.log 2>&1; rc=$?
tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o leg \
  -- python3 bench.py --only spmv_shapes --no-cpu > $OUT/shapes.json 2> $OUT/prof.err || exit 1
python3 -c "
import json; s=json.loads(open('$OUT/shapes.json').read().splitlines()[-1])
print(' '.join(f\"{k} {s[k]['kernel']} cold {s[k]['cold_kernel_ms']*1e3:.2f} us frac {s[k]['frac']}\" for k in ('cant','rma10','powerlaw')))"
grep -i "fixup\|spmv_tile" $OUT/prof/leg_kernel_stats.csv | cut -d, -f1-4
