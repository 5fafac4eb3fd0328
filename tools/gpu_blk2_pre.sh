#!/bin/bash
# GPU: two-camera last-frame parity tests on the in-tree library, then the Tracking-harness A/B
# (tools/gpu_enum_ab.sh over variants_lat/*).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_matcher.py \
  tests/test_capi_consumer.py -k "lastframe or two_cams or kb8 or tracking" > gpurun_out/b2pre_tests.log 2>&1 || { tail -30 gpurun_out/b2pre_tests.log; exit 1; }
tail -1 gpurun_out/b2pre_tests.log
bash tools/gpu_enum_ab.sh
