set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02h
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02h/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r02h/pytest.log; [ $rc -le 1 ] || exit $rc
for b in 1 0; do MSPMV_SPMV_BLOCKS=$b timeout -k 10 300 python tools/lab/narrow_probe.py || exit $?; done
