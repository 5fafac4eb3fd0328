#!/bin/bash
# GPU: rocprofv3 kernel-trace summaries of the matcher benchmarks, kept under profiles/: the Tracking
# thread's matcher calls (bench.matcher_calls) and config 5 at N = 1000 / 5000 (bench.matcher_config5_n).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/mprof
mkdir -p $D
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/calls -o run -- python3 -c "import json,bench; r = bench.matcher_calls(20); print(json.dumps(r['calls']))" > $D/calls.log 2>&1 || { tail -20 $D/calls.log; exit 1; }
for n in 1000 5000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c5_$n -o run -- python3 -c "import json,bench; r = bench.matcher_config5_n(10, $n); print(json.dumps(r['per_th']))" > $D/c5_$n.log 2>&1 || { tail -20 $D/c5_$n.log; exit 1; }
done
for f in calls c5_1000 c5_5000; do cp $(find $D/$f -name '*kernel_stats.csv' | head -1) $D/${f}_kernel_stats.csv; grep '^{' $D/$f.log | cut -c1-300; done
