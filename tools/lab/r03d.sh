#!/bin/bash
# r03d: k_spmm_blk one-wave workgroups (MSPMV_SPMM_BLK_TB=64) vs 256-thread tiles, PB 2 / 4
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03d; mkdir -p $OUT
T=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so
for i in 1 2; do
  for v in "tree256:$T:256" "tree64:$T:64" "pb4_256:$PWD/tools/lab/libmspmv_pb4.so:256" "pb4_64:$PWD/tools/lab/libmspmv_pb4.so:64"; do
    n=${v%%:*}; r=${v#*:}; lib=${r%:*}; tb=${r##*:}
    MSPMV_LIB=$lib MSPMV_SPMM_BLK_TB=$tb timeout -k 10 180 python tools/lab/spmm_cold_probe.py > $OUT/${n}_$i.json 2>$OUT/${n}_$i.err || { echo "$n rc=$?"; tail -3 $OUT/${n}_$i.err; exit 1; }
    echo "$n $i $(cat $OUT/${n}_$i.json)"
  done
done
