#!/bin/bash
# Cold timing: read-sweep flush (default) vs the old write sweep, spmv_shapes + spmm16 legs.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02n; mkdir -p $O
for mode in read write; do
  for leg in spmv_shapes spmm16; do
    MSPMV_FLUSH=$mode timeout -k 10 300 python bench.py --only $leg --no-cpu > $O/${leg}_$mode.json 2>$O/${leg}_$mode.err || exit $?
    echo "$mode $leg $(cut -c1-900 $O/${leg}_$mode.json)"
  done
done
