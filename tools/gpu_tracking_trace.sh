#!/bin/bash
# GPU: kernel + copy trace of the drop-in Tracking frame (tests/native/capi_frontend --tracking over the
# bench's seeded stereo sequence), summarised per kernel and as one frame's GPU timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/tracking_trace
mkdir -p $D
python3 tools/dropin_job.py $D/job.bin 60
timeout -k 10 60 tests/native/capi_frontend --tracking 60 $D/job.bin || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $D -o run -- tests/native/capi_frontend --tracking 60 $D/job.bin > $D/log 2>&1 || { tail -20 $D/log; exit 1; }
tail -1 $D/log
python3 tools/dropin_timeline.py $D --frame-after "k_sbp_block<0>" > $D/timeline.txt
cat $D/timeline.txt
rm -rf $D/*/ $D/*.csv $D/job.bin
