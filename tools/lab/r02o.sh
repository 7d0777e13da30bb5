#!/bin/bash
# Tile-kernel LDS trim (18.5 KB: 8 workgroups/CU): GPU parity suite, then the CG single leg on the
# tree build (92 VGPRs, 5 waves) vs lab builds compiled for 7 / 8 waves (spilling), then the bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest_gpu.log | head -20; exit $rc; }
for i in 1 2; do
  for v in tree cgw7 cgw8; do
    if [ $v = tree ]; then lib=$PWD/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so; else lib=$PWD/tools/lab/libmspmv_$v.so; fi
    MSPMV_LIB=$lib timeout -k 10 300 python bench.py --only cg_single --no-cpu > $O/cg_${v}_$i.json 2>$O/cg_${v}_$i.err || exit $?
    python -c "import json;d=json.load(open('$O/cg_${v}_$i.json'));print('$v', d['iterations'], d['us_per_iter'], d['roofline_frac'])"
  done
done
timeout -k 10 600 python bench.py --no-cpu > $O/bench.json 2>$O/bench.err || exit $?
python - <<'PY'
import json
d=json.load(open('gpurun_out/r02o/bench.json'))
print('headline', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])
for k,v in d.get('spmv_shapes',{}).items(): print(k, v['hot_kernel_ms'], v['cold_kernel_ms'], v['frac'])
print('nlpkkt', d['spmv_nlpkkt120_size'])
print('cg_multi', d['cg_multi']['ms_per_iter'], d['cg_multi']['roofline_frac'])
PY
