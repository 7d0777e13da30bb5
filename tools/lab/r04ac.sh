#!/bin/bash
# r04ac: the tree with L = 16 tiles of 32 items per lane group and its own plan key -- the full GPU
# suite, then the SpMM shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04ac; mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -rf > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -4 $OUT/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 tools/lab/spmm_probe.py > $OUT/spmm.json 2>$OUT/spmm.err; echo "probe rc=$?"; cat $OUT/spmm.json
