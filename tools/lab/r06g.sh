#!/bin/bash
# r06g: the pipelined single-RHS CG on the offset windows (k_cg1_dia): parity, then the pwtk-size CG in its
# forms (windows U = 8 / U = 4 offsets per batch, split) and a kernel trace of the windows form.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06g; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_cg.py tests/test_gpu_cg_resident.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
probe() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python tools/lab/cg_large_probe.py > $OUT/cgl_$name.json 2>$OUT/cgl_$name.err || { echo "cgl $name rc=$?"; tail -3 $OUT/cgl_$name.err; return 1; }
  echo "$name $(cat $OUT/cgl_$name.json)"
}
for i in 1 2; do
  probe pipe8_$i MSPMV_CG_RESIDENT=0 || exit 1
  probe pipe4_$i MSPMV_CG_RESIDENT=0 MSPMV_CG1_DIA_U=4 || exit 1
  probe split_$i MSPMV_CG_RESIDENT=0 MSPMV_CG_SPLIT=1 || exit 1
done
MSPMV_CG_RESIDENT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_pipe -o cgl -- python3 tools/lab/cg_large_probe.py > $OUT/prof_pipe.json 2>$OUT/prof_pipe.err || { echo "prof rc=$?"; tail -3 $OUT/prof_pipe.err; exit 1; }
echo done
