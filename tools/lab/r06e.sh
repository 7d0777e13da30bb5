#!/bin/bash
# r06e: one-generation tile fill for small single-RHS matrices (cant, rma10; MSPMV_SPMV_FILL=0 = nominal
# tiles) A/B + parity; the pwtk-size single CG: pipelined vs split (windows) forms, and a trace of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06e; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_spmv.py tests/test_gpu_blocks.py tests/test_gpu_split_rows.py tests/test_gpu_cg.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2 3; do
  for f in 0 1; do
    MSPMV_SPMV_FILL=$f timeout -k 10 300 python bench.py --only spmv_shapes --no-cpu > $OUT/shapes_f${f}_$i.json 2>$OUT/shapes_f${f}_$i.err || { echo "shapes rc=$?"; tail -3 $OUT/shapes_f${f}_$i.err; exit 1; }
    echo "fill=$f $i $(python -c "import json;d=json.load(open('$OUT/shapes_f${f}_$i.json'));print([(k, d[k]['cold_kernel_ms'], d[k]['frac']) for k in ('cant','rma10')])")"
  done
done
for i in 1 2; do
  MSPMV_CG_RESIDENT=0 timeout -k 10 300 python tools/lab/cg_large_probe.py > $OUT/cgl_pipe_$i.json 2>$OUT/cgl_pipe_$i.err || { echo "cgl rc=$?"; tail -3 $OUT/cgl_pipe_$i.err; exit 1; }
  cat $OUT/cgl_pipe_$i.json
  MSPMV_CG_RESIDENT=0 MSPMV_CG_SPLIT=1 timeout -k 10 300 python tools/lab/cg_large_probe.py > $OUT/cgl_split_$i.json 2>$OUT/cgl_split_$i.err || { echo "cgl rc=$?"; tail -3 $OUT/cgl_split_$i.err; exit 1; }
  cat $OUT/cgl_split_$i.json
done
MSPMV_CG_RESIDENT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_pipe -o cgl -- python3 tools/lab/cg_large_probe.py > $OUT/prof_pipe.json 2>$OUT/prof_pipe.err || { echo "prof rc=$?"; tail -3 $OUT/prof_pipe.err; exit 1; }
MSPMV_CG_RESIDENT=0 MSPMV_CG_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_split -o cgl -- python3 tools/lab/cg_large_probe.py > $OUT/prof_split.json 2>$OUT/prof_split.err || { echo "prof rc=$?"; tail -3 $OUT/prof_split.err; exit 1; }
find $OUT -name "*kernel_stats.csv"
