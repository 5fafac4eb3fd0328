#!/bin/bash
# GPU: extractor parity suite on the in-tree library, then kernel-trace A/B of variants/liborbfe_*.so
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_extractor.py \
  tests/test_gpu_batch.py tests/test_gpu_opencv_model.py > gpurun_out/fast_tests.log 2>&1 || { tail -30 gpurun_out/fast_tests.log; exit 1; }
tail -1 gpurun_out/fast_tests.log
REPS=${REPS:-2} bash tools/gpu_variants_trace.sh
