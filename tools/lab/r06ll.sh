#!/bin/bash
# r06ll: phase stamps of the sliced-ELL SpMV (lab library with -DMSPMV_SELL_LAB_STAMPS) on the power-law leg and the
# scattered band.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06ll; mkdir -p $OUT
export TMPDIR=/tmp
MSPMV_LIB=$PWD/tools/lab/libmspmv_sellstamps.so timeout -k 10 300 python3 -u tools/lab/sell_stamps.py > $OUT/stamps.jsonl 2>$OUT/stamps.err || { echo "rc=$?"; tail -5 $OUT/stamps.err; exit 1; }
cat $OUT/stamps.jsonl
