# GPU: extractor parity with the default build, then each variants/*.so benched (describe A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_extractor.py -x -q > gpurun_out/tq.log 2>&1 || { tail -30 gpurun_out/tq.log; exit 1; }
tail -2 gpurun_out/tq.log
bash tools/gpu_variants.sh
