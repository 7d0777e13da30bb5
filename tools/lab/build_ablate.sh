#!/bin/bash
# Lab builds of libmspmv.so with compile-time ablations of the SpMV tile kernel (measurement only;
# results are wrong by construction).  MSPMV_LIB=tools/lab/libmspmv_ablN.so selects one.
#   (the MSPMV_LAB_ABLATE switches are added to the kernels by hand for an experiment and removed after)
set -e
cd "$(dirname "$0")/../.."
C=sparse-matrix-linear-equations_amd/csrc
make -s -C $C -j8 >/dev/null
for n in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden -fopenmp \
     -Iinclude -DMSPMV_LAB_ABLATE=$n -c $C/mspmv_kernels.hip -o /tmp/abl_$n.o &
done
wait
for n in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/lab/libmspmv_abl$n.so /tmp/abl_$n.o \
     $C/build/mspmv_api.o $C/build/mspmv_dist.o $C/build/mspmv_cg_resident.o $C/build/mspmv_synth.o $C/build/mspmv_io.o $C/build/mspmv_spai.o $C/build/mspmv_ic0.o \
     -fopenmp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
