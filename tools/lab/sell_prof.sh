#!/bin/bash
# The power-law variant's SpMV under rocprofv3 --kernel-trace --stats, one run per MSPMV_SPMV_SLAB value
# (SELL_MODES; '' = the default plan, 4 = the sliced-ELL column groups).  The r05ao-r05ap ablations ran
# this with MSPMV_SELL_LAB bits of a lab build (phases skipped) that the kernel no longer has.
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05ap}
mkdir -p "$OUT"
for M in ${SELL_MODES:-default 4}; do
  P=$M; [ "$M" = default ] && P=""
  PROBE_ONLY=powerlaw PROBE_MODES="$P" timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/prof_$M" -o run -- python3 -u tools/lab/slab_group_probe.py > "$OUT/probe_$M.log" 2>&1
done
