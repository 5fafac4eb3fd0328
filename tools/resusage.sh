#!/bin/bash
# Per-kernel VGPR / LDS / occupancy of liborbfe's device code (compile-only, no GPU).
# usage: tools/resusage.sh [kernels.hip variant] [extra hipcc flags...]
cd "$(dirname "$0")/../orb_slam3_ros_amd/csrc"
K=${1:-orbfe_kernels.hip}; shift
if [ "$K" != orbfe_kernels.hip ]; then
  cp "$K" _exp_kernels.hip
  sed 's/#include "orbfe_kernels.hip"/#include "_exp_kernels.hip"/' orbfe_engine.hip > _exp_engine.hip
  SRC=_exp_engine.hip
else
  SRC=orbfe_engine.hip
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -c -o /tmp/_ru.o $SRC "$@" \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import sys,re
name=None
for l in sys.stdin:
    m=re.search(r"Function Name: (\S+)",l)
    if m: name=m.group(1); continue
    for key in ("VGPRs:","ScratchSize","Occupancy","LDS Size"):
        if key in l and name and ("k_" in name):
            print(name[:40], l.split("remark:")[1].rsplit(" [-Rpass",1)[0].strip())
' | grep -E "${KFILTER:-.}"
rm -f _exp_kernels.hip _exp_engine.hip
