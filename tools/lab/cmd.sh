set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_ic0.py tests/test_gpu_tools.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tic.log 2>&1; rc=$?; tail -2 gpurun_out/tic.log; [ $rc -eq 0 ] || exit $rc
for t in 0 1; do echo "tagged=$t $(MSPMV_TRSV_TAGGED=$t timeout -k 10 300 python tools/pcg_probe.py 8 20 | cut -c 1-600)" || exit 1; done
