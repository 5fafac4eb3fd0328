#!/bin/bash
# GPU: LDS bank-conflict share (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE) and L2 hit rate per kernel
# for each variants/liborbfe_*.so on the default bench workload (one --pmc pass per counter group).
set -o pipefail
cd $GRAFT_REPO_ROOT
export ORBFE_LIB_PARTIAL=1   # A/B baselines built from older commits may predate entry points
export TMPDIR=/tmp
PCMD="python bench.py --frames 512 --steps 3 --warmup 1 --stage-steps 1 --no-cpu-baseline --no-parity --matcher-steps 0 --rectify-steps 0 --no-side-configs"
for so in variants/liborbfe_*.so; do
  n=$(basename $so .so)
  i=0
  for grp in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    D=gpurun_out/lds_${n}_$i
    ORBFE_LIB=$PWD/$so timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $D -o run -- $PCMD > $D.log 2>&1 || { tail -20 $D.log; exit 1; }
  done
  python3 - "$n" <<'PY'
import csv, glob, collections, sys
n = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"gpurun_out/lds_{n}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"].split("(")[0].replace("orbfe::", "")][r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(acc):
    c = acc[k]
    lds = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"] if c.get("SQ_LDS_IDX_ACTIVE") else None
    l2 = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]) if c.get("TCC_HIT_sum") else None
    print(f"{n:22s} {k:16s} lds_conflict_share {lds if lds is None else round(lds, 4)}  l2_hit {l2 if l2 is None else round(l2, 4)}")
PY
done
