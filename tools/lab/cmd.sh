set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_tools.py tests/test_gpu_spmv.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tt.log 2>&1; rc=$?; tail -3 gpurun_out/tt.log; ./sparse-matrix-linear-equations_amd/mspmv/bin/facade_demo; exit $rc
