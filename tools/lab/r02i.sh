set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02i
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02i/pytest.log 2>&1
rc=$?; tail -12 gpurun_out/r02i/pytest.log; [ $rc -le 1 ] || exit $rc
MSPMV_BENCH_SHARDED=1 timeout -k 10 300 python bench.py --no-cpu --no-cg --steps 200 > gpurun_out/r02i/sharded1.json 2>gpurun_out/r02i/sharded1.err || exit $?
cat gpurun_out/r02i/sharded1.json
