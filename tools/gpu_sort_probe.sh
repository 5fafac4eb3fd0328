#!/bin/bash
# GPU: k_debug_block_sort durations per array length for each variants/liborbfe_*.so.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp ORBFE_LIB_PARTIAL=1
for so in variants/liborbfe_*.so; do
  n=$(basename $so .so)
  D=gpurun_out/sp_$n
  ORBFE_LIB=$PWD/$so timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $D -o sp -- python3 tools/sort_probe.py 10 > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
  python3 - $D $n <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "debug_block_sort" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sizes = (40, 120, 300, 600, 1200, 2400)
out = []
for i, n in enumerate(sizes):
    d = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows[10 * i:10 * i + 10])
    out.append(f"{n}:{d[len(d) // 2]:.1f}")
print(sys.argv[2], "median us per n:", " ".join(out))
PY
  rm -rf $D
done
