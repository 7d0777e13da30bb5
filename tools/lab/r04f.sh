#!/bin/bash
# r04f: node-block tests + A/B: tree (per-lane adjacent pairs, lean kernel) vs r03 on pwtk / perturbed shapes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04f; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_blocks.py -m gpu -q -p no:cacheprovider -x > $OUT/blocks.txt 2>&1; rc=$?
tail -3 $OUT/blocks.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in tree r03; do
    if [ $v = tree ]; then lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; shapes="pwtk pwtk_odd pwtk_extra pwtk_perturbed"; else lib=$PWD/tools/lab/libmspmv_r03.so; shapes="pwtk"; fi
    MSPMV_LIB=$lib timeout -k 10 200 python3 tools/lab/spmv_probe.py $shapes > $OUT/${v}_$rep.txt 2>$OUT/${v}_$rep.err || { echo "$v rc=$?"; tail -3 $OUT/${v}_$rep.err; exit 1; }
    python3 -c "
import json,sys
for l in open('$OUT/${v}_$rep.txt'): d=json.loads(l); print('$v', $rep, d['shape'], d['kernel'], d['kernel_us'], d['frac'])"
  done
done
