set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cgprof -o cg -- python3 tools/cg_probe.py --child > gpurun_out/cgprof.txt 2>&1; rc=$?; tail -2 gpurun_out/cgprof.txt; exit $rc
