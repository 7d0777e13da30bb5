set -o pipefail
export TMPDIR=/tmp
PROBE_SHAPE=${PROBE_SHAPE:-nlpkkt} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$1 -o cg -- python3 tools/cg_probe.py --child > gpurun_out/$1.txt 2>&1; rc=$?; grep "{" gpurun_out/$1.txt; exit $rc
