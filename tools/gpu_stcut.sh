#!/bin/bash
# GPU: stereo parity (extractor / batch / frame / C-ABI consumer tests) with the fused median cut,
# then batch-1 frame latency of the tree against variants_lat/* (tools/gpu_dropin_trace.sh's loop) and
# a short bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_extractor.py \
  tests/test_gpu_batch.py tests/test_capi_consumer.py tests/test_gpu_opencv_model.py > gpurun_out/stcut_tests.log 2>&1 || { tail -30 gpurun_out/stcut_tests.log; exit 1; }
tail -1 gpurun_out/stcut_tests.log
python3 tools/dropin_job.py /tmp/job.bin
for rep in 1 2 3; do
  echo -n "tree "; timeout -k 10 60 tests/native/capi_frontend --latency 200 /tmp/job.bin | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['frame_call']['frame_ms'], d['frame_call']['split_ms'])" || exit 1
  for d in variants_lat/*/; do
    echo -n "$(basename $d) "; LD_LIBRARY_PATH=$PWD/$d:$LD_LIBRARY_PATH timeout -k 10 60 tests/native/capi_frontend --latency 200 /tmp/job.bin | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['frame_call']['frame_ms'], d['frame_call']['split_ms'])" || exit 1
  done
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --matcher-steps 0 --rectify-steps 0 --no-side-configs --dropin-frames 0 > gpurun_out/stcut_bench.json 2> gpurun_out/stcut_bench.err || { tail -20 gpurun_out/stcut_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/stcut_bench.json')); print(d['value'], d['stage_ms'], d['parity']['ok'])"
