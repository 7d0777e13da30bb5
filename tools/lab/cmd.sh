set -o pipefail
MSPMV_LIB=$PWD/tools/lab/libmspmv_new.so timeout -k 10 400 python -u -m pytest tests/test_gpu_cg.py tests/test_gpu_dist.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do for v in head new; do echo "$v $(MSPMV_LIB=$PWD/tools/lab/libmspmv_$v.so PROBE_SHAPE=nlpkkt timeout -k 10 200 python tools/cg_probe.py --child | cut -c 60-250)" || exit 1; done; done
