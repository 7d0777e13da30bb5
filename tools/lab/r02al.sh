#!/bin/bash
# Row ends issued with the stream (MSPMV_SPMV_EARLY_RE=1) vs after the staging (0): SpMV tests with
# the knob on, then the striped-kernel shapes (cant, rma10, nlpkkt120 size) and the single CG.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02al; mkdir -p $O
MSPMV_SPMV_EARLY_RE=1 timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_spmv.py tests/test_gpu_cg.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    MSPMV_SPMV_EARLY_RE=$v timeout -k 10 300 python bench.py --only spmv_shapes --no-cpu > $O/s_${v}_$i.json 2> $O/s_${v}_$i.err || exit 1
    MSPMV_SPMV_EARLY_RE=$v timeout -k 10 120 python tools/cg_probe.py --child > $O/c_${v}_$i.json 2> $O/c_${v}_$i.err || exit 1
    MSPMV_SPMV_EARLY_RE=$v timeout -k 10 300 python bench.py --only cg_multi --no-cpu > $O/n_${v}_$i.json 2> $O/n_${v}_$i.err || exit 1
    python3 - <<PY
import json
s=json.load(open("$O/s_${v}_$i.json")); c=json.load(open("$O/c_${v}_$i.json")); n=json.load(open("$O/n_${v}_$i.json"))
print("early=$v", {k:(v2["hot_kernel_ms"], v2["cold_kernel_ms"]) for k,v2 in s.items() if isinstance(v2, dict) and "hot_kernel_ms" in v2},
      "parabolic spmv", c["spmv_kernel_us"], "cg", c["cg_us_per_iter"], "nlpkkt spmv", n["spmv_nlpkkt120_size"]["kernel_ms"])
PY
  done
done
