#!/bin/bash
# Collect PMC counter passes (one rocprofv3 run per pass, --kernel-trace only, no tracing
# domains) for a command.  Per run at most 8 SQ_, 4 TCC_, 4 TCP_, 2 TA_, 2 TD_, 2 GRBM_ counters.   usage: tools/pmc_passes.sh OUTDIR KERNEL_REGEX -- cmd...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=$1; RE=$2; shift 3
mkdir -p "$OUT"
export TMPDIR=/tmp
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
  "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM"
  "TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TOTAL_CACHE_ACCESSES"
  "TCC_HIT TCC_MISS TCC_EA0_RDREQ TCC_REQ"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES"
  "TA_DATA_STALLED_BY_TC_CYCLES TA_FLAT_READ_WAVEFRONTS"
)
i=0
for p in "${PASSES[@]}"; do
  timeout -k 10 300 rocprofv3 --pmc $p --kernel-trace --kernel-include-regex "$RE" --output-format csv \
      -d "$OUT/pass$i" -o p -- "$@" > "$OUT/pass$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc ($p)"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pass$i.log"; [ $rc -eq 1 ] || exit $rc; fi
  i=$((i+1))
done
