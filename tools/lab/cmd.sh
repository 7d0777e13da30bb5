set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_spmv.py tests/test_gpu_cg.py tests/test_spai.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tc16.log 2>&1; rc=$?; tail -3 gpurun_out/tc16.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for c in 0 1; do
  for L in 8; do echo "nlpkkt c16=$c L=$L $(MSPMV_SPMV_C16=$c SWEEP_SHAPE=nlpkkt SWEEP_L=$L SWEEP_BATCH=1 timeout -k 10 200 python tools/spmv_sweep.py --child | cut -c 1-400)" || exit 1; done
  for L in 4 16; do echo "fem c16=$c L=$L $(MSPMV_SPMV_C16=$c SWEEP_L=$L timeout -k 10 200 python tools/spmv_sweep.py --child | cut -c 1-400)" || exit 1; done
done; done
for c in 0 1; do echo "cg c16=$c $(MSPMV_SPMV_C16=$c PROBE_SHAPE=nlpkkt timeout -k 10 300 python tools/cg_probe.py --child 2>&1 | tail -2 | cut -c 1-600)" || exit 1; done
