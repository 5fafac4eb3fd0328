#!/bin/bash
# GPU: k_remap kernel time (trace) and HBM traffic (FETCH_SIZE, WRITE_SIZE passes) of the bench's
# rectification leg for each variants/liborbfe_*.so (ORBFE_LIB).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CMD="python bench.py --steps 1 --warmup 1 --stage-steps 0 --no-cpu-baseline --no-parity --matcher-steps 0 --no-side-configs --rectify-steps 3"
for so in variants/liborbfe_*.so; do
  n=$(basename $so .so)
  D=gpurun_out/rmp_$n
  mkdir -p $D
  ORBFE_LIB=$PWD/$so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D/t -o run -- $CMD > $D/t.log 2>&1 || { tail -5 $D/t.log; exit 1; }
  ORBFE_LIB=$PWD/$so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $D/f -o run -- $CMD > $D/f.log 2>&1 || { tail -5 $D/f.log; exit 1; }
  ORBFE_LIB=$PWD/$so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $D/w -o run -- $CMD > $D/w.log 2>&1 || { tail -5 $D/w.log; exit 1; }
  python - "$D" "$n" <<'PY'
import csv, glob, sys
d, n = sys.argv[1], sys.argv[2]
t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(glob.glob(d + "/t/**/*kernel_trace.csv", recursive=True)[0])) if "k_remap" in r["Kernel_Name"]]
def pmc(sub, name):
    v = {}
    for r in csv.DictReader(open(glob.glob(d + "/" + sub + "/**/*counter_collection.csv", recursive=True)[0])):
        if "k_remap" in r["Kernel_Name"] and r["Counter_Name"] == name:
            v[r["Dispatch_Id"]] = v.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return sorted(v.values())[len(v) // 2] * 1024
f, w = pmc("f", "FETCH_SIZE"), pmc("w", "WRITE_SIZE")
print(f"{n:20s} k_remap {sorted(t)[len(t)//2]:7.1f} us  fetch raw {f/1e6:7.1f} MB (x2 {2*f/1e6:7.1f})  write {w/1e6:7.1f} MB  per launch")
PY
done
