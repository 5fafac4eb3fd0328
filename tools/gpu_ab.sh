#!/bin/bash
# GPU: the extractor / batch parity tests on the working tree's library, then the kernel-trace A/B
# of every variants/liborbfe_*.so (tools/gpu_variants_trace.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_batch.py tests/test_gpu_opencv_model.py tests/test_gpu_getters.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
REPS=${REPS:-2} bash tools/gpu_variants_trace.sh
