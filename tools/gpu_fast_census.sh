#!/bin/bash
# GPU: the k_fast census (tools/fast_census.py builds variants/liborbfe_fast{1..5}.so): per variant the
# isolated k_fast time (kernel trace of a short bench run, every launch in stream order) and its
# VALU / LDS instruction counts (one rocprofv3 --pmc pass).
set -o pipefail
cd $GRAFT_REPO_ROOT
export ORBFE_LIB_PARTIAL=1
export TMPDIR=/tmp
PCMD="python bench.py --frames 512 --steps 3 --warmup 1 --stage-steps 1 --no-cpu-baseline --no-parity --matcher-steps 0 --rectify-steps 0 --no-side-configs --dropin-frames 0"
for so in variants/liborbfe_fast*.so; do
  n=$(basename $so .so)
  D=gpurun_out/fc_${n}
  ORBFE_LIB=$PWD/$so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- $PCMD > $D.log 2>&1 || { tail -20 $D.log; exit 1; }
  echo "=== $n"
  python3 tools/trace_grid_summary.py $D | grep -E "k_fast|k_resize" || true
  P=gpurun_out/fp_${n}
  ORBFE_LIB=$PWD/$so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SALU --kernel-include-regex k_fast --output-format csv -d $P -o run -- $PCMD > $P.log 2>&1 || { tail -20 $P.log; exit 1; }
  python3 - "$P" <<'PY'
import csv, glob, collections, sys
acc = collections.defaultdict(float); disp = set()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r.get("Dispatch_Id"))
# per launch group of 1024 images: the bench runs warmup + steps + stage steps passes of 3 k_fast launches
print("  pmc", {k: round(v / max(len(disp) / 3, 1) / 1e6, 2) for k, v in sorted(acc.items())}, "M per pass,", len(disp), "dispatches")
PY
  rm -rf $D $P
done
