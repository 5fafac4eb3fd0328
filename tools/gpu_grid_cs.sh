#!/bin/bash
# GPU: matcher / backend parity (every grid and band index build), then the matcher-call and config-5
# kernel traces (k_mt_grid's counting sort).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_matcher.py \
  tests/test_gpu_backend.py tests/test_capi.py tests/test_capi_consumer.py > gpurun_out/grid_tests.log 2>&1 || { tail -30 gpurun_out/grid_tests.log; exit 1; }
tail -1 gpurun_out/grid_tests.log
tools/gpu_matcher_calls_trace.sh && grep '^{' gpurun_out/mc_trace.log
bash tools/gpu_config5_trace.sh
