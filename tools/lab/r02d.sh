set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_spmv.py tests/test_gpu_cg.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02d/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r02d/pytest.log; [ $rc -le 1 ] || exit $rc
for cfg in "0 1" "0 0" "1638 1" "1638 0" "1792 1" "1536 1" "0 1"; do
  set -- $cfg
  MSPMV_SPMV_TILE=$1 MSPMV_SPMV_BLOCKS=$2 timeout -k 10 300 python bench.py --no-cpu --no-cg --no-extras --steps 400 > gpurun_out/r02d/b_$1_$2.json 2>gpurun_out/r02d/b_$1_$2.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/r02d/b_$1_$2.json'));print('tile=$1 blocks=$2', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
