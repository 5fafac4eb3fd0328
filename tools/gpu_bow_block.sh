set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_matcher.py tests/test_gpu_backend.py > gpurun_out/bow_tests.log 2>&1 || { tail -30 gpurun_out/bow_tests.log; exit 1; }
tail -2 gpurun_out/bow_tests.log
tools/gpu_matcher_calls_trace.sh
