#!/bin/bash
# r06a: the fold-ticket guard (GPU tests incl. the poisoned-ticket cases and the round-5 mechanism), the
# workgroup window SpMM / fused block-CG p update, windows plus a remainder; then A/B on the legs that
# take tickets and windows: base = round-5 library, wave = this tree with MSPMV_DIA_WG=0, tree = this tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06a; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_faults.py tests/test_gpu_dia.py tests/test_gpu_cg.py tests/test_gpu_dist.py tests/test_gpu_split_rows.py tests/test_gpu_slab.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log; grep "mechanism" $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; exit 1; }
TREE=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so
BASE=$PWD/tools/lab/libmspmv_r05.so
timeout -k 10 300 python bench.py --only window_shapes --no-cpu > $OUT/window_shapes.json 2>$OUT/window_shapes.err || { echo "window_shapes rc=$?"; tail -5 $OUT/window_shapes.err; exit 1; }
cat $OUT/window_shapes.json
for i in 1 2; do
  for v in base wave tree; do
    lib=$TREE; ev="MSPMV_X=1"
    [ $v = base ] && lib=$BASE
    [ $v = wave ] && ev="MSPMV_DIA_WG=0"
    for leg in cg_multi spmv_shapes; do
      env $ev MSPMV_LIB=$lib timeout -k 10 300 python bench.py --only $leg --no-cpu > $OUT/${leg}_${v}_$i.json 2>$OUT/${leg}_${v}_$i.err || { echo "$leg $v rc=$?"; tail -3 $OUT/${leg}_${v}_$i.err; exit 1; }
    done
    env $ev MSPMV_LIB=$lib timeout -k 10 300 python bench.py --steps 100 --no-cpu --no-extras --no-cg > $OUT/head_${v}_$i.json 2>$OUT/head_${v}_$i.err || { echo "head $v rc=$?"; exit 1; }
    echo "$v $i $(python -c "import json;d=json.load(open('$OUT/cg_multi_${v}_$i.json'));print(d['ms_per_iter'],d['roofline_frac'],d['iterations'],d['spmv_nlpkkt120_size']['kernel_ms'])") $(python -c "import json;d=json.load(open('$OUT/head_${v}_$i.json'));print(d['roofline']['frac'])") $(python -c "import json;d=json.load(open('$OUT/spmv_shapes_${v}_$i.json'));print(d['powerlaw']['frac'], d['cant']['frac'], d['rma10']['frac'])" | cut -c1-80)"
  done
done
timeout -k 10 300 python tools/tile_stamps.py > $OUT/tile_stamps.jsonl 2>$OUT/tile_stamps.err || { echo "stamps rc=$?"; tail -3 $OUT/tile_stamps.err; exit 1; }
echo stamps done
