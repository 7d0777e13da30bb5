set -o pipefail
PROBE_VARIANTS=8:48,16:48,7:48,6:48,4:48 timeout -k 10 500 python tools/cg_probe.py > gpurun_out/cgprobe_ipt.txt 2>&1; rc=$?; cat gpurun_out/cgprobe_ipt.txt; exit $rc
