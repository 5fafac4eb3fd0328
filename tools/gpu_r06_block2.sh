# GPU: two-camera last-frame searches (k_sbp_block2 and the multi-launch fallback) against the
# oracle, the KB8 Tracking harness parity, then the KB8 Tracking frame timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_matcher.py tests/test_capi_consumer.py -x -q --timeout 200 --timeout-method thread -m gpu -k "two_cams or kb8 or lastframe or rig or sbp_local or pose" > gpurun_out/b2_tests.log 2>&1 || { tail -40 gpurun_out/b2_tests.log; exit 1; }
tail -2 gpurun_out/b2_tests.log
python -c "import bench; bench.write_sequence_job('/tmp/kb8.bin', 60, 512, 512, 1000, 20, 31, (256.0, 256.0))"
timeout -k 10 120 tests/native/capi_frontend --tracking-kb8 60 /tmp/kb8.bin /tmp/kb8.out > gpurun_out/kb8_track.json 2> gpurun_out/kb8_track.err || { tail -20 gpurun_out/kb8_track.err; exit 1; }
tail -c 1500 gpurun_out/kb8_track.json
