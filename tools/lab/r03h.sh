#!/bin/bash
# r03h: k_spmm_blk new defaults vs next-chunk prefetch (PF) at 8 / 7 waves, one-wave workgroups; stamps
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03h; mkdir -p $OUT
bash tools/lab/ab_libs.sh $OUT 2 tools/lab/spmm_cold_probe.py tree libmspmv_pf.so libmspmv_pfw7.so || exit 1
for i in 1 2; do MSPMV_SPMM_BLK_TB=64 timeout -k 10 180 python tools/lab/spmm_cold_probe.py > $OUT/tb64_$i.json 2>$OUT/tb64_$i.err || exit 1; echo "tb64 $i $(cat $OUT/tb64_$i.json)"; done
MSPMV_LIB=$PWD/tools/lab/libmspmv_stamps10.so timeout -k 10 200 python tools/lab/stamps_blk.py > $OUT/stamps.json 2>$OUT/stamps.err
