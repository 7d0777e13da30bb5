set -o pipefail
for r in 1 2; do for v in head new; do echo "$v $(MSPMV_LIB=$PWD/tools/lab/libmspmv_$v.so SWEEP_ROUNDS=1 SWEEP_VARIANTS=8:1:0:0:48 timeout -k 10 200 python tools/spmv_sweep.py | cut -c 150-300)" || exit 1; done; done
for sh in parabolic; do for v in head new; do echo "$v $(MSPMV_LIB=$PWD/tools/lab/libmspmv_$v.so PROBE_SHAPE=$sh timeout -k 10 200 python tools/cg_probe.py --child | cut -c 60-250)" || exit 1; done; done
