set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02c
for cfg in "2048 1" "1638 1" "1638 0" "1792 1" "1536 1" "1365 1" "1170 1" "2048 1"; do
  set -- $cfg
  MSPMV_SPMV_TILE=$1 MSPMV_SPMV_BLOCKS=$2 timeout -k 10 300 python bench.py --no-cpu --no-cg --no-extras --steps 400 > gpurun_out/r02c/b_$1_$2.json 2>gpurun_out/r02c/b_$1_$2.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/r02c/b_$1_$2.json'));print('tile=$1 blocks=$2', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
