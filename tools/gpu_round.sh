# GPU: full parity suite, the default bench line, rocprofv3 kernel-trace stats of the bench command.
# Optional: PMC=1 adds the per-kernel counter passes (tools/gpu_profile_round.sh, isolated-timing build).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-parity --matcher-steps 0 ${BENCH_ARGS} > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
echo stats ok
if [ -n "$PMC" ]; then PREFIX=${PREFIX:-r03} bash tools/gpu_profile_round.sh; fi
