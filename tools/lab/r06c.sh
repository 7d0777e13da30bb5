#!/bin/bash
# r06c: the wave window SpMM at L = 8 with 5 / 6 waves per SIMD forced (spills) vs the default; configs[4]'s
# CG with the p update fused into the wave window SpMM vs the separate pass (MSPMV_DIA_PUPD=0) vs round 5;
# parity of the window and CG paths.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06c; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_dia.py tests/test_gpu_cg.py tests/test_gpu_faults.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
  for w in 0 5 6; do
    MSPMV_DIA_WPE=$w PROBE_L="8" PROBE_ONLY=nlpkkt timeout -k 10 300 python tools/lab/dia_probe.py > $OUT/probe_wpe${w}_$i.json 2>$OUT/probe_wpe${w}_$i.err || { echo "probe rc=$?"; tail -3 $OUT/probe_wpe${w}_$i.err; exit 1; }
    echo "wpe=$w $(cat $OUT/probe_wpe${w}_$i.json)"
  done
done
TREE=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so
BASE=$PWD/tools/lab/libmspmv_r05.so
for i in 1 2; do
  for v in base sep fused; do
    lib=$TREE; ev="MSPMV_X=1"
    [ $v = base ] && lib=$BASE
    [ $v = sep ] && ev="MSPMV_DIA_PUPD=0"
    env $ev MSPMV_LIB=$lib timeout -k 10 300 python bench.py --only cg_multi --no-cpu > $OUT/cg_multi_${v}_$i.json 2>$OUT/cg_multi_${v}_$i.err || { echo "cg $v rc=$?"; tail -3 $OUT/cg_multi_${v}_$i.err; exit 1; }
    echo "$v $i $(python -c "import json;d=json.load(open('$OUT/cg_multi_${v}_$i.json'));print(d['ms_per_iter'],d['roofline_frac'],d['iterations'])")"
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 600 --timeout-method thread > $OUT/pytest_full.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest_full.log | head -20; tail -5 $OUT/pytest_full.log; exit 1; }
tail -2 $OUT/pytest_full.log
