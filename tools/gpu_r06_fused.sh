# GPU: SearchLocalPoints with isInFrustum fused into the one-workgroup searches: the matcher and
# Tracking-harness parity tests, then both harnesses' timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_matcher.py tests/test_capi_consumer.py tests/test_gpu_extractor.py -x -q --timeout 200 --timeout-method thread -m gpu -k "local or frustum or track or kb8 or device_view or rig or pose or lastframe" > gpurun_out/fused_tests.log 2>&1 || { tail -40 gpurun_out/fused_tests.log; exit 1; }
tail -2 gpurun_out/fused_tests.log
python -c "import bench; bench.write_sequence_job('/tmp/seq.bin', 60); bench.write_sequence_job('/tmp/kb8.bin', 60, 512, 512, 1000, 20, 31, (256.0, 256.0))"
timeout -k 10 120 tests/native/capi_frontend --tracking 60 /tmp/seq.bin /tmp/trk.out > gpurun_out/trk.json 2> gpurun_out/trk.err || { tail -20 gpurun_out/trk.err; exit 1; }
tail -c 700 gpurun_out/trk.json
timeout -k 10 120 tests/native/capi_frontend --tracking-kb8 60 /tmp/kb8.bin /tmp/kb8.out > gpurun_out/kb8t.json 2> gpurun_out/kb8t.err || { tail -20 gpurun_out/kb8t.err; exit 1; }
tail -c 700 gpurun_out/kb8t.json
