# GPU: the fisheye kNN in both block shapes (batched / few frames) against the oracle, then the KB8
# Tracking harness (one-frame kNN inside orbfe_frame_fisheye).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_extractor.py tests/test_gpu_batch.py tests/test_gpu_matcher.py tests/test_distributed.py tests/test_capi_consumer.py -x -q --timeout 200 --timeout-method thread -m gpu -k "fisheye or knn or rig or kb8" > gpurun_out/knn_tests.log 2>&1 || { tail -30 gpurun_out/knn_tests.log; exit 1; }
tail -2 gpurun_out/knn_tests.log
python -c "import bench; bench.write_sequence_job('/tmp/kb8.bin', 60, 512, 512, 1000, 20, 31, (256.0, 256.0))"
timeout -k 10 120 tests/native/capi_frontend --tracking-kb8 60 /tmp/kb8.bin /tmp/kb8.out > gpurun_out/kb8t.json 2> gpurun_out/kb8t.err || { tail -20 gpurun_out/kb8t.err; exit 1; }
tail -c 500 gpurun_out/kb8t.json
