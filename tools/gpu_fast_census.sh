#!/bin/bash
# GPU: per-phase census of one kernel across the variants/liborbfe_*.so ablation builds (the
# -DORBFE_ABLATE_FAST=N ladder: 1 staging, 2 + pass 1, 3 + entries / pass 2, 4 + NMS / emission
# without the minTh fallback, 0 full). One rocprofv3 --pmc pass (instruction counts, wave cycles)
# with its kernel trace per variant; prints per-variant totals per bench step.
# usage: KREGEX=k_fast bash tools/gpu_fast_census.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export ORBFE_LIB_PARTIAL=1   # A/B baselines built from older commits may predate entry points
export TMPDIR=/tmp
K=${KREGEX:-k_fast}
PCMD="python bench.py --frames 512 --steps 3 --warmup 1 --stage-steps 1 --no-cpu-baseline --no-parity --matcher-steps 0 --rectify-steps 0 --no-side-configs"
for so in variants/liborbfe_*.so; do
  n=$(basename $so .so)
  D=gpurun_out/census_${n}
  rm -rf $D
  ORBFE_LIB=$PWD/$so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$K" --kernel-trace --output-format csv -d $D -o run -- $PCMD > $D.log 2>&1 || { tail -20 $D.log; exit 1; }
  python3 - "$n" "$D" "$K" <<'PY'
import csv, glob, collections, sys
n, d, k = sys.argv[1:4]
acc = collections.defaultdict(float)
disp = set()
dur = 0.0
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if k not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        disp.add(r.get("Dispatch_Id"))
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if k in r["Kernel_Name"]:
            dur += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
steps = 4   # warmup 1 + steps 3, one stage step excluded below when present
print(n, f"dispatches={len(disp)}", f"dur_us_total={dur:.1f}", " ".join(f"{key}={val:.5g}" for key, val in sorted(acc.items())))
PY
done
