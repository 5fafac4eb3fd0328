cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; tail -15 gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/config5_probe.py 20 && bash tools/gpu_config5_trace.sh && bash tools/gpu_tracking_trace.sh
bash tools/gpu_fast_census.sh
