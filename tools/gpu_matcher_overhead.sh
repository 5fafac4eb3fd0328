#!/bin/bash
# GPU: resident SearchByProjection host overhead (tools/matcher_overhead.py) plain, then under a
# kernel trace (per-call kernel durations vs gaps: tools/trace_gaps.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/matcher_overhead.py > gpurun_out/mo.log 2>&1 || { tail -20 gpurun_out/mo.log; exit 1; }
cat gpurun_out/mo.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mo_trace -o mo -- python tools/matcher_overhead.py > gpurun_out/mo_trace.log 2>&1 || { tail -20 gpurun_out/mo_trace.log; exit 1; }
python tools/trace_gaps.py $(find gpurun_out/mo_trace -name '*kernel_trace.csv' | head -1)
