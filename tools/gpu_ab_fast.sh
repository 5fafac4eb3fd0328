#!/bin/bash
# GPU: extractor + batched-path parity on the in-tree library, then REPS kernel-trace A/B rounds
# over variants/liborbfe_*.so (tools/gpu_variants_trace.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
bash tools/gpu_variants_trace.sh
