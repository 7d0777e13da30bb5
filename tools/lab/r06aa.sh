#!/bin/bash
# r06aa: planar {r, p} buffers for the windows pipelined CG (whole-line writes): CG / resident / fault tests, then
# the pwtk-size pipelined CG (35.3-35.8 us per iteration interleaved: r06z, r06w) x3 and its kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06aa; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_cg.py tests/test_gpu_cg_resident.py tests/test_gpu_faults.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2 3; do
  MSPMV_CG_RESIDENT=0 timeout -k 10 300 python tools/lab/cg_large_probe.py > $OUT/cgl_$i.json 2>$OUT/cgl_$i.err || { echo "rc=$?"; tail -3 $OUT/cgl_$i.err; exit 1; }
  cat $OUT/cgl_$i.json
done
MSPMV_CG_RESIDENT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o cgl -- python3 tools/lab/cg_large_probe.py > $OUT/prof.json 2>$OUT/prof.err || { echo "prof rc=$?"; tail -3 $OUT/prof.err; exit 1; }
MSPMV_CG_RESIDENT=0 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o cgl -- python3 tools/lab/cg_large_probe.py > $OUT/pmcw.json 2>$OUT/pmcw.err || { echo "pmc rc=$?"; tail -3 $OUT/pmcw.err; exit 1; }
echo done
