#!/bin/bash
# per-level k_pyrfast durations (kernel trace) for each library in VARIANTS
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/lv
for v in ${VARIANTS}; do
  n=$(basename $v .so)
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lv/$n -o run -- python tools/pf_time.py $v > gpurun_out/lv/$n.log 2>&1 || { tail -5 gpurun_out/lv/$n.log; exit 1; }
  echo "== $n"; python tools/pf_trace_summary.py gpurun_out/lv/$n | grep -E "per level|k_fallback|k_pyrfast|k_fast |k_resize"
done
