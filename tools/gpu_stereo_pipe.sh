# GPU: k_stereo two-stage pipeline A/B: the product build's stereo parity tests, then kernel traces of
# variants/liborbfe_{base,stp}.so on the bench workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_batch.py tests/test_capi_consumer.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/stp_tests.log 2>&1 || { tail -30 gpurun_out/stp_tests.log; exit 1; }
tail -2 gpurun_out/stp_tests.log
REPS=2 bash tools/gpu_variants_trace.sh 2>&1 | grep -E "===|k_stereo"
