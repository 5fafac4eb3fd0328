#!/bin/bash
# GPU: the Tracking-frame harness with the current frame read in HBM (orbfe_frame_device_view, the
# product path) against the host-copy form (--tracking-hostview), 3 alternating runs each, plus the
# CPU twin's parity of both (same per-frame slots).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python3 tools/dropin_job.py gpurun_out/seq.bin 60 || exit 1
timeout -k 10 300 tests/native/tracking_cpu 60 gpurun_out/seq.bin gpurun_out/cpu.out > gpurun_out/trk_cpu.json || exit 1
for r in 1 2 3; do
  for mode in --tracking --tracking-hostview; do
    timeout -k 10 120 tests/native/capi_frontend $mode 60 gpurun_out/seq.bin gpurun_out/gpu.out > gpurun_out/trk.json || exit 1
    same=$(cmp -s gpurun_out/gpu.out gpurun_out/cpu.out && echo parity_ok || echo MISMATCH)
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/trk.json').read().strip().splitlines()[-1]); print(sys.argv[1], d['tracking_frame_ms'], d['split_ms'], sys.argv[2])" $mode $same
  done
done
