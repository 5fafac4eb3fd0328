#!/bin/bash
# GPU: parity of each variants/liborbfe_*.so on the extractor + batch tests (ORBFE_LIB override),
# then the kernel-trace A/B of all of them (tools/gpu_variants_trace.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export ORBFE_LIB_PARTIAL=1   # A/B baselines built from older commits may predate entry points
mkdir -p gpurun_out
for so in variants/liborbfe_*.so; do
  v=$(basename $so .so)
  ORBFE_LIB=$PWD/$so timeout -k 10 300 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/ab_$v.log 2>&1 || { tail -30 gpurun_out/ab_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/ab_$v.log)"
done
REPS=${REPS:-2} bash tools/gpu_variants_trace.sh
