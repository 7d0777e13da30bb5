#!/bin/bash
# r05j: the whole -m gpu suite on the current tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05j; mkdir -p $OUT
timeout -k 10 1150 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || grep -E "Error|assert |FAILED" $OUT/pytest.log | head -20
exit $rc
