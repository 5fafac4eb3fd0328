#!/bin/bash
# Builds the k_describe LDS-DMA A/B variants (r05_kernel_ab.txt item 14) from a patched copy of the
# sources (the product kernel carries no A/B hooks): variants/liborbfe_dma{6,5,4}.so, the number
# being the waves-per-SIMD target. Run on the GPU with scratch-style bench lines per ORBFE_LIB.
set -e
cd "$(dirname "$0")/.."
T=$(mktemp -d)
cp -r orb_slam3_ros_amd include "$T/"
(cd "$T" && patch -p1 -s < "$OLDPWD/tools/describe_dma.patch")
mkdir -p variants
for w in 6 5 4; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math \
    -DDP_DMA -DDP_WAVES=$w -o variants/liborbfe_dma$w.so "$T/orb_slam3_ros_amd/csrc/orbfe_engine.hip" &
done
wait
rm -rf "$T"
