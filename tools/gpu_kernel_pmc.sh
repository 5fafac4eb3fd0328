#!/bin/bash
# GPU: one kernel's issue / LDS / scalar counters for each variants/liborbfe_*.so (one rocprofv3 --pmc
# pass per group, --kernel-include-regex), summed per variant. usage: KREGEX=k_fast bash tools/gpu_kernel_pmc.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export ORBFE_LIB_PARTIAL=1   # A/B baselines built from older commits may predate entry points
export TMPDIR=/tmp
K=${KREGEX:-k_fast}
PCMD="python bench.py --frames 512 --steps 2 --warmup 1 --stage-steps 1 --no-cpu-baseline --no-parity --matcher-steps 0 --rectify-steps 0 --no-side-configs"
for so in variants/liborbfe_*.so; do
  n=$(basename $so .so)
  i=0
  for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU" \
             "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_UNALIGNED_STALL SQ_INST_LEVEL_LDS SQ_WAVES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    D=gpurun_out/kp_${n}_$i
    ORBFE_LIB=$PWD/$so timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$K" --kernel-trace --output-format csv -d $D -o run -- $PCMD > $D.log 2>&1 || { tail -20 $D.log; exit 1; }
  done
  python3 - "$n" <<'PY'
import csv, glob, collections, sys
n = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(f"gpurun_out/kp_{n}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("orbfe::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((f, r.get("Dispatch_Id")))
for k in sorted(acc):
    c = acc[k]
    print(n, k, " ".join(f"{key}={val:.4g}" for key, val in sorted(c.items())))
PY
done
