#!/bin/bash
# r04ag: the tree with three streaming workgroups per CU in the CG -- the GPU suite, then configs[4].
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04ag; mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -rf > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -4 $OUT/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do timeout -k 10 200 python3 tools/lab/cgmulti_probe.py; done
