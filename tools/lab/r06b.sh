#!/bin/bash
# r06b: tickets released only in the few-block folds (k_fold_dot, split rows); the workgroup window
# SpMM vs the wave form (plain L = 8 / 16 on the nlpkkt120 size); configs[4]'s CG: base (round 5),
# wave (MSPMV_DIA_WG=0: no fused p update), tree; a kernel trace of the tree's CG leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06b; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_faults.py tests/test_gpu_slab.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
TREE=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so
BASE=$PWD/tools/lab/libmspmv_r05.so
for i in 1 2; do
  for v in 0 1; do
    MSPMV_DIA_WG=$v PROBE_L="8 16" PROBE_ONLY=nlpkkt timeout -k 10 300 python tools/lab/dia_probe.py > $OUT/probe_wg${v}_$i.json 2>$OUT/probe_wg${v}_$i.err || { echo "probe rc=$?"; tail -3 $OUT/probe_wg${v}_$i.err; exit 1; }
    echo "wg=$v $(cat $OUT/probe_wg${v}_$i.json)"
  done
done
for i in 1 2; do
  for v in base wave tree; do
    lib=$TREE; ev="MSPMV_X=1"
    [ $v = base ] && lib=$BASE
    [ $v = wave ] && ev="MSPMV_DIA_WG=0"
    env $ev MSPMV_LIB=$lib timeout -k 10 300 python bench.py --only cg_multi --no-cpu > $OUT/cg_multi_${v}_$i.json 2>$OUT/cg_multi_${v}_$i.err || { echo "cg $v rc=$?"; tail -3 $OUT/cg_multi_${v}_$i.err; exit 1; }
    env $ev MSPMV_LIB=$lib timeout -k 10 300 python bench.py --only spmv_shapes --no-cpu > $OUT/spmv_shapes_${v}_$i.json 2>$OUT/spmv_shapes_${v}_$i.err || { echo "shapes $v rc=$?"; exit 1; }
    echo "$v $i $(python -c "import json;d=json.load(open('$OUT/cg_multi_${v}_$i.json'));print(d['ms_per_iter'],d['roofline_frac'],d['iterations'])") $(python -c "import json;d=json.load(open('$OUT/spmv_shapes_${v}_$i.json'));print(d['powerlaw']['frac'], d['cant']['frac'], d['rma10']['frac'])")"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_cg -o cg -- python bench.py --only cg_multi --no-cpu > $OUT/prof_cg.log 2>&1 || { echo "rocprof rc=$?"; tail -5 $OUT/prof_cg.log; exit 1; }
find $OUT/prof_cg -name "*kernel_stats.csv" | head -3
