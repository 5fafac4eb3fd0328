#!/bin/bash
# Round-2 GPU pass: full parity suite, default bench line, kernel-trace stats of the bench command,
# then per-path VALU / wait / LDS counters (tools/gpu_prof_pf.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu ${TEST_ARGS} > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -3 gpurun_out/tests.log
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
[ -n "${NO_PROF}" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-parity --matcher-steps 0 ${BENCH_ARGS} > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
bash tools/gpu_prof_pf.sh
