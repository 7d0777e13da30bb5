#!/bin/bash
# r04c: SpMV A/B (round-3 library vs tree) on the bench shapes + perturbation breakdown, then bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
OUT=gpurun_out/r04c; mkdir -p $OUT
export TMPDIR=/tmp
R03=$PWD/tools/lab/libmspmv_r03.so
timeout -k 10 300 python3 tools/lab/spmv_probe.py > $OUT/probe_tree1.txt 2>$OUT/probe_tree1.err || { echo "tree1 rc=$?"; tail -5 $OUT/probe_tree1.err; exit 1; }
cat $OUT/probe_tree1.txt
MSPMV_LIB=$R03 timeout -k 10 300 python3 tools/lab/spmv_probe.py pwtk nlpkkt cant powerlaw scatter > $OUT/probe_r03.txt 2>$OUT/probe_r03.err || { echo "r03 rc=$?"; tail -5 $OUT/probe_r03.err; exit 1; }
cat $OUT/probe_r03.txt
timeout -k 10 300 python3 tools/lab/spmv_probe.py pwtk pwtk_perturbed nlpkkt > $OUT/probe_tree2.txt 2>$OUT/probe_tree2.err || { echo "tree2 rc=$?"; exit 1; }
cat $OUT/probe_tree2.txt
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2>$OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
