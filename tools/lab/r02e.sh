set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_spmv.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02e/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r02e/pytest.log; [ $rc -le 1 ] || exit $rc
for cfg in "1 1" "1 0" "0 0" "1 1" "1 0"; do
  set -- $cfg
  MSPMV_SPMV_BLOCKS=$1 MSPMV_SPMV_BLKREG=$2 timeout -k 10 300 python bench.py --no-cpu --no-cg --no-extras --steps 400 > gpurun_out/r02e/b_$1_$2.json 2>gpurun_out/r02e/b_$1_$2.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/r02e/b_$1_$2.json'));r=d['roofline'];print('blocks=$1 blkreg=$2', d['value'], r['kernel'], r['kernel_ms'], r['frac'])"
done
