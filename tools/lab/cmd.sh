set -o pipefail
for r in 1 2; do for v in base prod abl10; do
  lib=tools/lab/libmspmv_$v.so; [ $v = prod ] && lib=sparse-matrix-linear-equations_amd/mspmv/libmspmv.so
  echo "fem $v $(MSPMV_LIB=$lib timeout -k 10 200 python tools/spmv_sweep.py --child | cut -c 150-330)" || exit 1
done; done
for v in base prod abl10; do
  lib=tools/lab/libmspmv_$v.so; [ $v = prod ] && lib=sparse-matrix-linear-equations_amd/mspmv/libmspmv.so
  echo "nlp $v $(MSPMV_LIB=$lib SWEEP_SHAPE=nlpkkt SWEEP_L=1 SWEEP_BATCH=1 timeout -k 10 200 python tools/spmv_sweep.py --child | cut -c 150-330)" || exit 1
  echo "cg1 $v $(MSPMV_LIB=$lib timeout -k 10 200 python tools/cg_probe.py --child 2>&1 | tail -1 | cut -c 1-300)" || exit 1
done
MSPMV_LIB=tools/lab/libmspmv_abl9.so timeout -k 10 200 python tools/lab/stamps.py > gpurun_out/stamps_fem2.json
