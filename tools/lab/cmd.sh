set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_ic0.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_ic0.log 2>&1; rc=$?; tail -15 gpurun_out/t_ic0.log; exit $rc
