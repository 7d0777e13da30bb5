#!/bin/bash
# r06z: iterations per graph batch (MSPMV_CG_BATCH) for the pwtk-size pipelined single CG: the host inspects batch b
# while b + 1 runs, so up to 2K - 1 launches run past convergence.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06z; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for k in def 4 2 16; do
    if [ $k = def ]; then E="MSPMV_DUMMY=0"; else E="MSPMV_CG_BATCH=$k"; fi
    env $E MSPMV_CG_RESIDENT=0 timeout -k 10 300 python tools/lab/cg_large_probe.py > $OUT/k_${k}_$i.json 2>$OUT/k_${k}_$i.err || { echo "rc=$?"; tail -3 $OUT/k_${k}_$i.err; exit 1; }
    echo "K=$k $(python -c "import json;d=json.load(open('$OUT/k_${k}_$i.json'));print(d['us_per_iter'], d['iterations'])")"
  done
done
echo done
