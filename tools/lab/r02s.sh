#!/bin/bash
# SQ stall counters for the SpMM (spmm16 leg), CG single and CG multi legs (one --pmc pass each).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02s; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS"
for leg in spmm16 cg_single cg_multi; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/$leg -o pmc -- python3 bench.py --only $leg --no-cpu > $O/$leg.json 2> $O/$leg.err
  rc=$?; echo "$leg rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$leg.err; exit $rc; }
done
