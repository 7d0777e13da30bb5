#!/bin/bash
# r03q: which resource bounds the generic tile SpMV on the nlpkkt120-size 27-point matrix (1.2 GB per
# launch)?  Knob sensitivity, alternating, one process per run: default, int32 columns (+2 B/nnz, same
# instruction count), one-wave tiles, row ends with the stream, merge walk everywhere, and the
# pair-load lab build (half the stream's load instructions, same bytes) -- after its parity tests.
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03q; mkdir -p $OUT
PAIR=$PWD/tools/lab/libmspmv_pair.so
MSPMV_LIB=$PAIR timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_gpu_spmv.py > $OUT/pair_tests.log 2>&1; rc=$?
tail -3 $OUT/pair_tests.log; [ $rc -eq 0 ] || exit $rc
MSPMV_SPMV_DICT=100 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_gpu_spmv.py -k "not test_column_dictionary_tiles" > $OUT/dict_tests.log 2>&1; rc=$?
tail -3 $OUT/dict_tests.log; [ $rc -eq 0 ] || exit $rc
export SWEEP_SHAPE=nlpkkt SWEEP_BATCH=1
for r in 1 2; do
  for v in "X=0" "MSPMV_LIB=$PAIR" "MSPMV_SPMV_C16=0" "MSPMV_SPMV_TB=64" "MSPMV_SPMV_DICT=100" "MSPMV_SPMV_RG_COST=0"; do
    env $v timeout -k 10 200 python tools/spmv_sweep.py --child > $OUT/run.json 2>$OUT/run.err || { echo "$v failed"; tail -3 $OUT/run.err; exit 1; }
    echo "$r ${v##*/} $(cat $OUT/run.json)"
  done
done
