#!/bin/bash
# GPU: kernel trace of tools/blk_probe.py for each variants/liborbfe_*.so (ORBFE_LIB), per-kernel means.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export ORBFE_LIB_PARTIAL=1
for so in variants/liborbfe_*.so; do
  n=$(basename $so .so)
  D=gpurun_out/bp_$n
  ORBFE_LIB=$PWD/$so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o bp -- python tools/blk_probe.py 30 > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
  echo "== $n $(tail -1 $D.log)"
  python3 - $D <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.reader(open(f)))[1:8]:
    print("  ", r[0][:36], r[1], round(float(r[3]) / 1e3, 2), "us")
PY
  rm -rf $D
done
