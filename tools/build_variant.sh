#!/bin/bash
# Build an experimental variant of the library: [TIMING_TOO=1] tools/build_variant.sh NAME "-DFLAG ..."
# -> gp-mpc_amd/gpmpc/lib/libgpmpc_mi355x_NAME.so (and _NAME_timing.so with the phase stamps); select it with
# GPMPC_LIB=... (its build id says "variant-NAME" and the flags; gpmpc/_lib.py checks only the in-tree default)
set -e
NAME=$1; DEFS=$2
cd "$(dirname "$0")/../gp-mpc_amd/csrc"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -mllvm -amdgpu-mfma-vgpr-form=1"
mkdir -p build/v_$NAME
TS=("")
[ -n "${TIMING_TOO:-}" ] && TS=("" timing)   # TIMING_TOO=1: also the phase-stamp build
for t in "${TS[@]}"; do
  T=""; [ "$t" = timing ] && T="-DGPMPC_TIMING"
  for s in sqp_kernel gp_kernels capi; do
    /opt/rocm/bin/hipcc $F $DEFS $T -c $s.hip -o build/v_$NAME/${s}${t}.o &
  done
  wait
  /opt/rocm/bin/hipcc -O2 -fPIC -DGPMPC_SRC_HASH="\"variant\"" -DGPMPC_GIT_HEAD="\"$(git rev-parse --short=12 HEAD)\"" \
      -DGPMPC_BUILD_KIND="\"variant-$NAME${t:+-$t} $DEFS\"" -c build_id.cpp -o build/v_$NAME/build_id${t}.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../gpmpc/lib/libgpmpc_mi355x_${NAME}${t:+_$t}.so \
      build/v_$NAME/sqp_kernel${t}.o build/v_$NAME/gp_kernels${t}.o build/v_$NAME/capi${t}.o build/v_$NAME/build_id${t}.o
done
