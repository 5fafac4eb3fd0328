#!/bin/bash
# GPU: k_pyramid duration (kernel trace of the drop-in latency run) per tile size (ORBFE_PYR_TILE; the
# knob is read only by a variant built with tools/build_variant.sh NAME -DORBFE_AB_KNOBS=1)
# and block size (variants/liborbfe_pyr{256,1024}.so via ORBFE_LIB; the in-tree library is 512).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
python3 tools/dropin_job.py gpurun_out/job.bin 40
run() {   # $1 label, $2 binary
  D=gpurun_out/pab_$1
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- $2 --latency 40 gpurun_out/job.bin > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
  python3 - $D $1 <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f)) if "k_pyramid" in r["Kernel_Name"])
print(sys.argv[2], "k_pyramid median us", round(d[len(d) // 2], 2) if d else None, "n", len(d))
PY
  rm -rf $D
}
for t in 80x64 64x48 48x40 112x80 160x100; do ORBFE_PYR_TILE=$t run nt512_$t tests/native/capi_frontend || exit 1; done
# a variant library beside a copy of the binary (it finds liborbfe.so by $ORIGIN/../../orb_slam3_ros_amd)
for nt in 256 1024; do
  V=gpurun_out/v$nt
  mkdir -p $V/tests/native $V/orb_slam3_ros_amd
  cp tests/native/capi_frontend $V/tests/native/ && cp variants/liborbfe_pyr$nt.so $V/orb_slam3_ros_amd/liborbfe.so
  for t in 80x64 48x40; do ORBFE_PYR_TILE=$t run nt${nt}_$t $V/tests/native/capi_frontend || exit 1; done
  rm -rf $V
done
rm -f gpurun_out/job.bin
