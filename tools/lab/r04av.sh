#!/bin/bash
# r04av: L = 8 row groups of one lane per column pair (Gp = 1) read their nonzeros' columns and values
# once per quad -- lane j reads nonzeros k + j and k + 4 + j, DPP quad broadcasts share them (dpp) --
# vs tree (every lane reads every nonzero from LDS), alternating: configs[4] CG and SpMM; then the
# SpMM parity tests on dpp.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04av; mkdir -p $OUT
bash tools/lab/ab_libs.sh $OUT/cg 2 tools/lab/cgmulti_probe.py tree libmspmv_dpp.so || exit 1
MSPMV_LIB=$PWD/tools/lab/libmspmv_dpp.so timeout -k 10 400 python -m pytest tests/test_gpu_spmv.py tests/test_gpu_split_rows.py tests/test_gpu_cg.py -m gpu -q -p no:cacheprovider -rf > $OUT/dpp_tests.log 2>&1
rc=$?; echo "dpp tests rc=$rc"; tail -3 $OUT/dpp_tests.log; exit $rc
