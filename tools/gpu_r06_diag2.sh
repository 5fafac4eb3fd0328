# GPU: the local-map search tests (multi-block passes, wide-window pass 0), the KB8 Tracking harness
# parity test, and the config-5 device times per th.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_matcher.py tests/test_capi_consumer.py -x -q --timeout 200 --timeout-method thread -m gpu -k "sbp_local or kb8" > gpurun_out/sbp_tests.log 2>&1 || { tail -30 gpurun_out/sbp_tests.log; exit 1; }
tail -2 gpurun_out/sbp_tests.log
timeout -k 10 200 python -u tools/matcher_ab.py 30 > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -20 gpurun_out/c5.err; exit 1; }
cat gpurun_out/c5.json
