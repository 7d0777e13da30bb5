#!/bin/bash
# r06f: split-CG vector passes with one pair per thread on short vectors (cg_update_blocks); the pwtk-size
# single CG in its forms (pipelined on windows / on tiles, split) with the plain SpMV beside each; configs[4]
# unchanged; a kernel trace of the pipelined-on-tiles and split forms.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_cg.py tests/test_gpu_dist.py tests/test_gpu_faults.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
probe() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python tools/lab/cg_large_probe.py > $OUT/cgl_$name.json 2>$OUT/cgl_$name.err || { echo "cgl $name rc=$?"; tail -3 $OUT/cgl_$name.err; return 1; }
  echo "$name $(cat $OUT/cgl_$name.json)"
}
for i in 1 2; do
  probe pipe_$i MSPMV_CG_RESIDENT=0 || exit 1
  probe pipe_tiles_$i MSPMV_CG_RESIDENT=0 MSPMV_DIA=0 || exit 1
  probe split_$i MSPMV_CG_RESIDENT=0 MSPMV_CG_SPLIT=1 || exit 1
done
timeout -k 10 300 python bench.py --only cg_multi --no-cpu > $OUT/cg_multi.json 2>$OUT/cg_multi.err || { echo "cg_multi rc=$?"; tail -3 $OUT/cg_multi.err; exit 1; }
head -c 600 $OUT/cg_multi.json; echo
MSPMV_CG_RESIDENT=0 MSPMV_DIA=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_pipe_tiles -o cgl -- python3 tools/lab/cg_large_probe.py > $OUT/prof_pipe_tiles.json 2>$OUT/prof_pipe_tiles.err || { echo "prof rc=$?"; tail -3 $OUT/prof_pipe_tiles.err; exit 1; }
MSPMV_CG_RESIDENT=0 MSPMV_CG_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_split -o cgl -- python3 tools/lab/cg_large_probe.py > $OUT/prof_split.json 2>$OUT/prof_split.err || { echo "prof rc=$?"; tail -3 $OUT/prof_split.err; exit 1; }
echo done
