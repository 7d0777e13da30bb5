#!/bin/bash
# r06l: L-wide window kernel loading each run's values two runs ahead (MSPMV_DIA_VPD=2; 4 waves per SIMD forced
# at L <= 8, 8 dwords spilled at L = 8) against one run ahead; parity under VPD=2, then the nlpkkt120-size SpMM per
# width and configs[4]'s CG, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06l; mkdir -p $OUT
export TMPDIR=/tmp
MSPMV_DIA_VPD=2 timeout -k 10 900 python -u -m pytest tests/test_gpu_dia.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
  for v in 1 2; do
    for L in 8 16 4; do
      MSPMV_DIA_VPD=$v PROBE_L=$L timeout -k 10 300 python tools/lab/spmm8_probe.py > $OUT/p_${v}_${L}_$i.json 2>$OUT/p_${v}_${L}_$i.err || { echo "probe rc=$?"; tail -3 $OUT/p_${v}_${L}_$i.err; exit 1; }
      echo "vpd=$v $(cat $OUT/p_${v}_${L}_$i.json)"
    done
    MSPMV_DIA_VPD=$v timeout -k 10 300 python bench.py --only cg_multi --no-cpu > $OUT/cgm_${v}_$i.json 2>$OUT/cgm_${v}_$i.err || { echo "cg_multi rc=$?"; tail -3 $OUT/cgm_${v}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/cgm_${v}_$i.json'));print('vpd=$v cg_multi', d['ms_per_iter'], d['roofline_frac'], d['iterations'])"
  done
done
echo done
