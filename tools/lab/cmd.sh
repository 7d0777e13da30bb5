set -o pipefail
export TMPDIR=/tmp
PROBE_SHAPE=nlpkkt timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cgm -o cgm -- python3 tools/cg_probe.py --child > gpurun_out/cgm.json 2>/dev/null || exit 1
cat gpurun_out/cgm.json; cut -d, -f1-5 gpurun_out/cgm/cgm_kernel_stats.csv | cut -c 1-150 | head -20
