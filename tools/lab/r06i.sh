#!/bin/bash
# r06i: masked offset windows summed without the mask selects first (exact rerun only for a non-finite row);
# MSPMV_DIA_EXACT=1 = the round-5 select form.  Parity, then configs[4] CG + nlpkkt120 SpMV and the pwtk-size
# single CG in both forms, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06i; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_dia.py tests/test_gpu_cg.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
  for ex in 0 1; do
    MSPMV_DIA_EXACT=$ex timeout -k 10 300 python bench.py --only cg_multi --no-cpu > $OUT/cgm_e${ex}_$i.json 2>$OUT/cgm_e${ex}_$i.err || { echo "cg_multi rc=$?"; tail -3 $OUT/cgm_e${ex}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/cgm_e${ex}_$i.json'));s=d['spmv_nlpkkt120_size'];print('exact=$ex', d['ms_per_iter'], d['roofline_frac'], d['iterations'], 'spmv', s['kernel_ms'], s['frac'])"
    MSPMV_DIA_EXACT=$ex MSPMV_CG_RESIDENT=0 timeout -k 10 300 python tools/lab/cg_large_probe.py > $OUT/cgl_e${ex}_$i.json 2>$OUT/cgl_e${ex}_$i.err || { echo "cgl rc=$?"; tail -3 $OUT/cgl_e${ex}_$i.err; exit 1; }
    echo "exact=$ex $(cat $OUT/cgl_e${ex}_$i.json)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cgm -o cgm -- python3 bench.py --only cg_multi --no-cpu > $OUT/prof_cgm.json 2>$OUT/prof_cgm.err || { echo "prof rc=$?"; tail -3 $OUT/prof_cgm.err; exit 1; }
echo done
