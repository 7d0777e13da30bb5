#!/bin/bash
# Lab builds of libmspmv.so with compile-time overrides (measurement A/B only):
#   tools/lab/build_variant.sh NAME "-DMACRO=VALUE ..."   ->  tools/lab/libmspmv_NAME.so
set -e
cd "$(dirname "$0")/../.."
C=sparse-matrix-linear-equations_amd/csrc
make -s -C $C -j8 >/dev/null
NAME=$1; DEFS=$2
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden -fopenmp \
   -Iinclude $DEFS -c $C/mspmv_kernels.hip -o /tmp/var_$NAME.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/lab/libmspmv_$NAME.so /tmp/var_$NAME.o \
   $C/build/mspmv_api.o $C/build/mspmv_dist.o $C/build/mspmv_cg_resident.o $C/build/mspmv_synth.o $C/build/mspmv_io.o $C/build/mspmv_spai.o $C/build/mspmv_ic0.o \
   -fopenmp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built tools/lab/libmspmv_$NAME.so"
