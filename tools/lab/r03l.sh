#!/bin/bash
# r03l: register-resident CG single -- parity tests, smoke, then the bench's cg_single leg both ways
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03l; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_cg_resident.py > $OUT/resident_tests.log 2>&1; rc=$?
tail -15 $OUT/resident_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_cg.py > $OUT/cg_tests.log 2>&1; rc=$?
tail -5 $OUT/cg_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
cat $OUT/smoke.log
for v in 1 0 1; do
  MSPMV_CG_RESIDENT=$v timeout -k 10 200 python bench.py --only cg_single --no-cpu > $OUT/cg_single_$v.json 2>$OUT/cg_single_$v.err || exit 1
  echo "resident=$v $(cat $OUT/cg_single_$v.json)"
done
