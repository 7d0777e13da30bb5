set -o pipefail
MSPMV_SPMV_TB=64 timeout -k 10 300 python -u -m pytest tests/test_gpu_spmv.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t64.log 2>&1; rc=$?; tail -3 gpurun_out/t64.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do for v in "256 8" "64 8" "64 16" "64 4"; do set -- $v; echo "tb=$1 ipt=$2 $(MSPMV_SPMV_TB=$1 SWEEP_ROUNDS=1 SWEEP_VARIANTS=$2:1:0:0:48 timeout -k 10 200 python tools/spmv_sweep.py | cut -c 150-330)" || exit 1; done; done
for v in "256 8" "64 8"; do set -- $v; echo "nlpkkt tb=$1 $(MSPMV_SPMV_TB=$1 MSPMV_SPMV_IPT=$2 SWEEP_SHAPE=nlpkkt SWEEP_L=1 SWEEP_BATCH=1 timeout -k 10 200 python tools/spmv_sweep.py --child | cut -c 150-330)" || exit 1; done
