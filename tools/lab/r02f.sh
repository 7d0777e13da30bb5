set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02f
for cfg in "8 0" "8 1792" "8 1536" "16 2560" "16 3072" "16 0" "8 0"; do
  set -- $cfg
  MSPMV_SPMV_IPT=$1 MSPMV_SPMV_TILE=$2 timeout -k 10 300 python bench.py --no-cpu --no-cg --no-extras --steps 400 > gpurun_out/r02f/b_$1_$2.json 2>gpurun_out/r02f/b_$1_$2.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/r02f/b_$1_$2.json'));r=d['roofline'];print('ipt=$1 tile=$2', d['value'], r['kernel'], r['kernel_ms'], r['frac'])"
done
