set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_tools.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -rf > gpurun_out/ttools.log 2>&1; rc=$?; tail -15 gpurun_out/ttools.log; exit $rc
