#!/bin/bash
# GPU: kernel trace of the batch-1 drop-in path (tests/native/capi_frontend --latency: two
# orbfe_extract threads + orbfe_stereo_match per frame through the host C-ABI), summarised per
# kernel and as one frame's GPU timeline (tools/dropin_timeline.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/dropin_trace
python3 tools/dropin_job.py gpurun_out/dropin_trace/job.bin
# latency, twice each: the in-tree library, then every variants_lat/<name>/liborbfe.so
# (LD_LIBRARY_PATH beats the RUNPATH)
for rep in 1 2; do
  echo -n "tree "
  timeout -k 10 60 tests/native/capi_frontend --latency 200 gpurun_out/dropin_trace/job.bin || exit 1
  for d in variants_lat/*/; do
    [ -f $d/liborbfe.so ] || continue
    echo -n "$(basename $d) "
    LD_LIBRARY_PATH=$PWD/$d:$LD_LIBRARY_PATH timeout -k 10 60 tests/native/capi_frontend --latency 200 gpurun_out/dropin_trace/job.bin || exit 1
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/dropin_trace -o run -- tests/native/capi_frontend --latency 60 gpurun_out/dropin_trace/job.bin > gpurun_out/dropin_trace/log 2>&1 || { tail -20 gpurun_out/dropin_trace/log; exit 1; }
tail -1 gpurun_out/dropin_trace/log
python3 tools/dropin_timeline.py gpurun_out/dropin_trace
# the raw traces exceed what gpurun copies back: keep the summaries only
rm -rf gpurun_out/dropin_trace/*/ gpurun_out/dropin_trace/*.csv gpurun_out/dropin_trace/job.bin
