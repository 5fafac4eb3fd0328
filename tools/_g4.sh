cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && timeout -k 10 400 python -u -m pytest tests/test_gpu_matcher.py tests/test_capi_consumer.py tests/test_gpu_extractor.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; tail -3 gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/config5_probe.py 20 > gpurun_out/c5.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/c5.txt; [ $rc -eq 0 ] || exit $rc
python3 tools/dropin_job.py gpurun_out/job.bin 60 && timeout -k 10 60 tests/native/capi_frontend --latency 100 gpurun_out/job.bin && timeout -k 10 60 tests/native/capi_frontend --tracking 60 gpurun_out/job.bin; rm -f gpurun_out/job.bin
bash tools/gpu_config5_trace.sh
