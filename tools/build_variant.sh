#!/bin/bash
# Build an experimental variant of the library: tools/build_variant.sh NAME "-DFLAG ..." [timing]
# -> gp-mpc_amd/gpmpc/lib/libgpmpc_mi355x_NAME.so (and _NAME_timing.so with the phase stamps)
set -e
NAME=$1; DEFS=$2
cd "$(dirname "$0")/../gp-mpc_amd/csrc"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -mllvm -amdgpu-mfma-vgpr-form=1"
mkdir -p build/v_$NAME
for t in "" timing; do
  T=""; [ "$t" = timing ] && T="-DGPMPC_TIMING"
  for s in sqp_kernel gp_kernels capi; do
    /opt/rocm/bin/hipcc $F $DEFS $T -c $s.hip -o build/v_$NAME/${s}${t}.o &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../gpmpc/lib/libgpmpc_mi355x_${NAME}${t:+_$t}.so \
      build/v_$NAME/sqp_kernel${t}.o build/v_$NAME/gp_kernels${t}.o build/v_$NAME/capi${t}.o
done
