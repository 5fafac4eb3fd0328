#!/bin/bash
# GPU: kernel trace of the bench's rectification leg (k_remap, 512 images) for each
# variants/liborbfe_*.so (ORBFE_LIB): mean k_remap duration and the leg's event time.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for so in variants/liborbfe_*.so; do
  n=$(basename $so .so)
  D=gpurun_out/rm_$n
  mkdir -p $D
  ORBFE_LIB=$PWD/$so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python bench.py --steps 2 --warmup 1 --stage-steps 0 --no-cpu-baseline --no-parity \
    --matcher-steps 0 --no-side-configs --rectify-steps 10 > $D/out.json 2> $D/err || { tail -5 $D/err; exit 1; }
  python - "$D" "$n" <<'PY'
import csv, glob, json, sys
d, n = sys.argv[1], sys.argv[2]
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f)) if "k_remap" in r["Kernel_Name"]]
leg = json.load(open(d + "/out.json"))["rectify_remap"]["ms_per_step"]
print(f"{n:24s} k_remap n={len(t)} mean={sum(t)/len(t):8.1f} us min={min(t):8.1f}  leg {leg} ms")
PY
done
