#!/bin/bash
# r06h: k_cg1_dia with the first batch's loads issued before the head (MSPMV_CG1_DIA_PRE=1, default) vs after.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06h; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cg.py -k "pipelined" -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
probe() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python tools/lab/cg_large_probe.py > $OUT/cgl_$name.json 2>$OUT/cgl_$name.err || { echo "cgl $name rc=$?"; tail -3 $OUT/cgl_$name.err; return 1; }
  echo "$name $(cat $OUT/cgl_$name.json)"
}
for i in 1 2 3; do
  probe pre1_$i MSPMV_CG_RESIDENT=0 || exit 1
  probe pre0_$i MSPMV_CG_RESIDENT=0 MSPMV_CG1_DIA_PRE=0 || exit 1
done
echo done
