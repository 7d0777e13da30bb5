set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_spmv.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tdict.log 2>&1; rc=$?; tail -2 gpurun_out/tdict.log; [ $rc -eq 0 ] || exit $rc
echo "band $(SWEEP_SHAPE=band SWEEP_BATCH=2 timeout -k 10 200 python tools/spmv_sweep.py --child | cut -c 180-330)" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bd -o bd -- python3 bench.py --no-cpu --no-cg --steps 20 > gpurun_out/bd.json 2>/dev/null || exit 1
grep -h "build_dict\|k_spmv_tile" gpurun_out/bd/*/bd_kernel_stats.csv gpurun_out/bd/bd_kernel_stats.csv 2>/dev/null | cut -c 1-160
