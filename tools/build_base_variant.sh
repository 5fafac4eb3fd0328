#!/bin/bash
# Build the committed HEAD's liborbfe.so into variants/ as the A/B baseline (git worktree in /tmp).
# usage: tools/build_base_variant.sh NAME [extra hipcc flags]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
wt=/tmp/orbfe_base_wt
[ -d $wt ] || git worktree add -f $wt HEAD >/dev/null
git -C $wt checkout -q --detach HEAD
git -C $wt reset -q --hard $(git rev-parse HEAD)
mkdir -p variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math \
  -Wno-unused-function "$@" -o variants/liborbfe_$name.so $wt/orb_slam3_ros_amd/csrc/orbfe_engine.hip
echo variants/liborbfe_$name.so
