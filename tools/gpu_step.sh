#!/bin/bash
# GPU: one round-5 check point: the GPU tests named in $TESTS (default: the whole -m gpu suite), then a
# short bench line (default workload, side legs off unless BENCH_ARGS says otherwise). Each step under its own time limit; the first failure ends
# the script.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
timeout -k 10 900 python -u -m pytest $TESTS -x -q -m gpu --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/tests.log 2>&1
rc=$?; tail -5 gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$EXTRA" ]; then
  timeout -k 10 600 bash -c "$EXTRA" > gpurun_out/extra.log 2>&1; rc=$?; tail -20 gpurun_out/extra.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:---steps 10 --warmup 3 --matcher-steps 10 --no-side-configs} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; tail -3 gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1]); print(json.dumps({k: d.get(k) for k in ('value','ms_per_step','stage_ms','dropin_latency_ms')})); print(json.dumps(d.get('dropin'))[:3000])"
fi
