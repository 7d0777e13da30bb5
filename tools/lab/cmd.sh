set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_spai.py tests/test_gpu_cg.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -15 gpurun_out/t.log; exit $rc
