#!/bin/bash
# GPU: BoW parity tests, then k_bow_block's phase stamps (variants/liborbfe_bowst.so, -DORBFE_BOW_STAMPS)
# on bench.matcher_calls, then the matcher_calls kernel trace of the product library.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_matcher.py \
  tests/test_gpu_backend.py -k "bow or BoW" > gpurun_out/bow_tests.log 2>&1 || { tail -30 gpurun_out/bow_tests.log; exit 1; }
tail -1 gpurun_out/bow_tests.log
ORBFE_LIB_PARTIAL=1 ORBFE_LIB=$PWD/variants/liborbfe_bowst.so timeout -k 10 120 python -c "import bench; bench.matcher_calls(5)" > gpurun_out/bowst.log 2>&1 || { tail -20 gpurun_out/bowst.log; exit 1; }
grep "^bow" gpurun_out/bowst.log | tail -4
tools/gpu_matcher_calls_trace.sh && grep '^{' gpurun_out/mc_trace.log
