set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_spmv.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tdict.log 2>&1; rc=$?; tail -4 gpurun_out/tdict.log; [ $rc -eq 0 ] || exit $rc
for d in 0 1; do
  echo "band dict=$d $(MSPMV_SPMV_DICT=$d SWEEP_SHAPE=band SWEEP_BATCH=2 timeout -k 10 200 python tools/spmv_sweep.py --child | cut -c 180-330)" || exit 1
done
