# GPU: block-search parity tests, then tools/blk_scale_probe.py on the product build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_matcher.py tests/test_capi_consumer.py -x -q --timeout 200 --timeout-method thread -m gpu -k "sbp or block or track or tracking or local" > gpurun_out/blk_tests.log 2>&1 || { tail -30 gpurun_out/blk_tests.log; exit 1; }
tail -2 gpurun_out/blk_tests.log
timeout -k 10 120 python tools/blk_scale_probe.py
