#!/bin/bash
# r05w: offset windows with paired value panels (16-B loads at L = 1) and the LDS-run L-wide kernel:
# parity, tiles vs windows on the probe shapes and on the configs[4] CG leg, then counter passes of the
# window and tile kernels on the nlpkkt120 size.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r05w; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dia.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; exit 1; }
MSPMV_DIA_RUNX=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_dia.py -x -q --timeout 120 --timeout-method thread -k "parity or forced or inf" > $OUT/pytest_runx.log 2>&1
rc=$?
tail -3 $OUT/pytest_runx.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest_runx.log | head -20; exit 1; }
bash tools/lab/ab_env.sh $OUT/ab 2 tools/lab/dia_probe.py "MSPMV_DIA=0" "MSPMV_DIA_SPMM=1" "MSPMV_DIA_SPMM=1 MSPMV_DIA_RUNX=1" || exit 1
bash tools/lab/ab_env.sh $OUT/cg 1 "bench.py --only cg_multi --no-cpu" "MSPMV_DIA_SPMM=0" "MSPMV_DIA_SPMM=1" || exit 1
timeout -k 10 700 bash tools/pmc_passes.sh $OUT/ctr "k_spmm_dia|k_spmm_tile|k_spmv_tile" -- python3 tools/lab/dia_ctr_probe.py || exit 1
python3 tools/counter_summary.py $OUT/ctr --title "r05w: offset windows vs merge tiles, nlpkkt120 size" > $OUT/counters.md
