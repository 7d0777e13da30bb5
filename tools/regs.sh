#!/bin/bash
# VGPR / SGPR / spill / LDS of the kernels in an in-tree HIP object (default: mspmv_kernels.o).
#   usage: tools/regs.sh [object.o] [name-substring ...]
set -eu
B=/opt/rocm/lib/llvm/bin
OBJ=${1:-sparse-matrix-linear-equations_amd/csrc/build/mspmv_kernels.o}
shift || true
T=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$OBJ"
$B/clang-offload-bundler --type=o --input=$T/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co --unbundle
$B/llvm-readelf --notes $T/k.co > $T/notes.txt
python3 "$(dirname "$0")/kernel_regs.py" $T/notes.txt "$@"
rm -rf "$T"
