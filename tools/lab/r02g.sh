set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02g
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02g/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r02g/pytest.log; [ $rc -le 1 ] || exit $rc
for b in 1 0; do
  MSPMV_SPMM_BLK=$b timeout -k 10 300 python bench.py --no-cpu --no-cg --steps 200 > gpurun_out/r02g/b_$b.json 2>gpurun_out/r02g/b_$b.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/r02g/b_$b.json'));s=d['spmm16'];print('spmm_blk=$b', d['value'], d['roofline']['frac'], 'pwtk', s['pwtk']['kernel_ms'], s['pwtk']['frac'], 'cant', s['cant']['kernel_ms'])"
done
