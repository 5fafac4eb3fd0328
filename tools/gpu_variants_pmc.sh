#!/bin/bash
# GPU: per-kernel VALU / SALU / LDS / wait counters of each variants/liborbfe_*.so (ORBFE_LIB).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CMD="python bench.py --steps 2 --warmup 1 --stage-steps 1 --no-cpu-baseline --no-parity --matcher-steps 0 --rectify-steps 0 --no-side-configs"
for so in variants/liborbfe_*.so; do
  n=$(basename $so .so)
  D=gpurun_out/vp_$n
  mkdir -p $D
  i=0
  for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"; do
    i=$((i+1))
    ORBFE_LIB=$PWD/$so timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $D/p$i -o run -- $CMD > $D/p$i.log 2>&1 || { tail -20 $D/p$i.log; exit 1; }
  done
  echo "=== $n"
  python tools/pf_pmc_summary.py $D | grep -A16 "^k_fast\|^k_resize"
done
