# GPU: k_fast dual-threshold pass 1 A/B: parity of the variant (extractor + batch tests), then kernel
# traces of variants/liborbfe_{base,dual}.so on the bench workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ORBFE_LIB_PARTIAL=1 ORBFE_LIB=$PWD/variants/liborbfe_dual.so timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_batch.py tests/test_gpu_opencv_model.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/dual_tests.log 2>&1 || { tail -30 gpurun_out/dual_tests.log; exit 1; }
tail -2 gpurun_out/dual_tests.log
REPS=2 bash tools/gpu_variants_trace.sh
