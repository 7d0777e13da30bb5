#!/bin/bash
# r03o: kernel traces of the split CG (nlpkkt120 size, L = 8), p.Ap pass vs SpMM dot mode (tail pass)
cd "$(dirname "$0")/../.."
OUT=$PWD/gpurun_out/r03o; mkdir -p $OUT; export TMPDIR=/tmp
for v in pass fused; do
  MSPMV_CG_DOT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o leg \
     -- python3 bench.py --only cg_multi --no-cpu > $OUT/$v.json 2> $OUT/$v.err || exit 1
  f=$(find $OUT/$v -name "*kernel_stats.csv" | head -1); echo "== $v"; cut -d, -f1-8 "$f" | head -12
done
