#!/bin/bash
# kernel timeline of the last pf_time.py batch (both paths) for the library $1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tl
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl/run -o run -- python tools/pf_time.py ${1:-orb_slam3_ros_amd/liborbfe.so} > gpurun_out/tl/log 2>&1 || { tail -5 gpurun_out/tl/log; exit 1; }
cat gpurun_out/tl/log | grep path
python tools/pf_timeline.py gpurun_out/tl/run
