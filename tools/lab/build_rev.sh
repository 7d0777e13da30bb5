#!/bin/bash
# A/B baseline library: libmspmv.so built from git revision REV into tools/lab/libmspmv_NAME.so
# (git-ignored; it travels to the GPU box with the tree), for tools/lab/ab_libs.sh.  Product code
# carries no lab switches: a variant is a revision.
#   usage: tools/lab/build_rev.sh REV NAME
set -eu
cd "$(dirname "$0")/../.."
REV=$1; NAME=$2
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
git archive "$REV" sparse-matrix-linear-equations_amd/csrc include | tar -x -C "$TMP"
mkdir -p "$TMP/sparse-matrix-linear-equations_amd/mspmv"
C=$TMP/sparse-matrix-linear-equations_amd/csrc
make -s -C "$C" -j8 "$C/../mspmv/libmspmv.so"
cp "$TMP/sparse-matrix-linear-equations_amd/mspmv/libmspmv.so" "tools/lab/libmspmv_$NAME.so"
echo "tools/lab/libmspmv_$NAME.so <- $REV"
