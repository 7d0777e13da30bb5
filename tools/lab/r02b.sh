set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02b
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_spmv.py tests/test_gpu_cg.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02b/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r02b/pytest.log; [ $rc -le 1 ] || exit $rc
for b in 0 1 0 1; do
  MSPMV_SPMV_BLOCKS=$b timeout -k 10 300 python bench.py --no-cpu --no-cg --no-extras --steps 400 > gpurun_out/r02b/bench_b$b.json 2>gpurun_out/r02b/bench_b$b.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/r02b/bench_b$b.json'));print('blocks=$b', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
