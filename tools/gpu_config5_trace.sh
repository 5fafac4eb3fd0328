#!/bin/bash
# GPU: kernel trace of device-resident config-5 searches at th 1 and 15 (tools/config5_trace.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for th in 1 15; do
  D=gpurun_out/c5_th$th
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/config5_trace.py $th 30 > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
  tail -1 $D.log
  python3 - $D <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.reader(open(f)))[1:12]:
    print("  ", r[0][:40], r[1], round(float(r[3]) / 1e3, 2), "us")
PY
  rm -rf $D
done
