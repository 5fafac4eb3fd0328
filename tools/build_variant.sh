#!/bin/bash
# Build an A/B variant of liborbfe.so into variants/ (compile-time flags), for tools/gpu_variants.sh.
# usage: tools/build_variant.sh NAME [extra hipcc flags, e.g. -DDP_KPW=1]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math \
  -Wno-unused-function "$@" -o variants/liborbfe_$name.so orb_slam3_ros_amd/csrc/orbfe_engine.hip
echo variants/liborbfe_$name.so
