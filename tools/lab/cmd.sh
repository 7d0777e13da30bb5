set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_spmv.py tests/test_gpu_cg.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do for c in 0 1; do echo "c16=$c $(MSPMV_SPMV_C16=$c SWEEP_ROUNDS=1 SWEEP_VARIANTS=8:1:0:0:48 timeout -k 10 200 python tools/spmv_sweep.py | cut -c 150-300)" || exit 1; done; done
for c in 0 1; do echo "c16=$c $(MSPMV_SPMV_C16=$c timeout -k 10 200 python tools/cg_probe.py --child | cut -c 60-250)" || exit 1; done
for c in 0 1; do echo "c16=$c $(MSPMV_SPMV_C16=$c SWEEP_SHAPE=nlpkkt SWEEP_L=1 SWEEP_BATCH=1 timeout -k 10 200 python tools/spmv_sweep.py --child | cut -c 150-300)" || exit 1; done
