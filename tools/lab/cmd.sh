set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_ic0.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_ic0.log 2>&1; rc=$?; tail -2 gpurun_out/t_ic0.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 500 python tools/pcg_probe.py 8 20 > gpurun_out/pcg_probe.txt 2>&1; rc=$?; tail -3 gpurun_out/pcg_probe.txt; exit $rc
