#!/bin/bash
# GPU: kernel trace of bench.matcher_calls (the Tracking thread's SearchForInitialization / SearchByBoW /
# SearchByProjection(F, KF) calls at their own sizes): per-kernel launch counts and mean durations.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/mc_trace
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 -c "import json,bench; r = bench.matcher_calls(20); print(json.dumps({k: (v['ms_per_call'], v['device_ms_per_call'], v['parity_ok']) for k, v in r['calls'].items()}))" > $D.log 2>&1 || { tail -20 $D.log; exit 1; }
tail -1 $D.log
python3 - $D <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.reader(open(f)))[1:25]:
    print("  ", r[0][:60], r[1], round(float(r[3]) / 1e3, 2), "us")
PY
