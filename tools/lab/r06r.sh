#!/bin/bash
# r06r: the scattered band on the sliced-ELL kernel with one column group (MSPMV_SPMV_SLAB=4 MSPMV_SLAB_GROUPS=1 / 2)
# against its default column-slab blocks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06r; mkdir -p $OUT
export TMPDIR=/tmp
probe() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python tools/lab/scatter_probe.py > $OUT/$name.json 2>$OUT/$name.err || { echo "$name rc=$?"; tail -3 $OUT/$name.err; return 1; }
  echo "$name $(cat $OUT/$name.json)"
}
for i in 1 2; do
  probe default_$i MSPMV_DUMMY=0 || exit 1
  probe sell_g1_$i MSPMV_SPMV_SLAB=4 MSPMV_SLAB_GROUPS=1 || exit 1
  probe sell_g2_$i MSPMV_SPMV_SLAB=4 MSPMV_SLAB_GROUPS=2 || exit 1
done
echo done
