#!/bin/bash
# r06k: the lane-per-row L-wide window kernel (MSPMV_DIA_RL=1) against the column-pair form: parity under RL=1,
# then the nlpkkt120-size SpMM per width and configs[4]'s CG, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r06k; mkdir -p $OUT
export TMPDIR=/tmp
MSPMV_DIA_RL=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_dia.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
  for rl in 0 1; do
    for L in 8 16 4 2; do
      MSPMV_DIA_RL=$rl PROBE_L=$L timeout -k 10 300 python tools/lab/spmm8_probe.py > $OUT/p_${rl}_${L}_$i.json 2>$OUT/p_${rl}_${L}_$i.err || { echo "probe rc=$?"; tail -3 $OUT/p_${rl}_${L}_$i.err; exit 1; }
      echo "rl=$rl $(cat $OUT/p_${rl}_${L}_$i.json)"
    done
    MSPMV_DIA_RL=$rl timeout -k 10 300 python bench.py --only cg_multi --no-cpu > $OUT/cgm_${rl}_$i.json 2>$OUT/cgm_${rl}_$i.err || { echo "cg_multi rc=$?"; tail -3 $OUT/cgm_${rl}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/cgm_${rl}_$i.json'));print('rl=$rl cg_multi', d['ms_per_iter'], d['roofline_frac'], d['iterations'])"
  done
done
echo done
