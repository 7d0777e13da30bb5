#!/bin/bash
# Lab library with the sliced-ELL kernel's phase stamps (mspmv_slab.hip built with -DMSPMV_SELL_LAB_STAMPS, every
# other object from the production build): tools/lab/libmspmv_sellstamps.so, for tools/lab/sell_stamps.py via MSPMV_LIB.
set -eu
cd "$(dirname "$0")/../.."
C=sparse-matrix-linear-equations_amd/csrc
make -C $C -j8 >/dev/null
mkdir -p /tmp/sellstamps
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden -fopenmp -Wall \
    -Wno-unused-function -Iinclude -DMSPMV_SELL_LAB_STAMPS -c $C/mspmv_slab.hip -o /tmp/sellstamps/mspmv_slab.o
OBJS=$(ls $C/build/*.o | grep -v mspmv_slab.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/lab/libmspmv_sellstamps.so $OBJS /tmp/sellstamps/mspmv_slab.o \
    -fopenmp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built tools/lab/libmspmv_sellstamps.so
