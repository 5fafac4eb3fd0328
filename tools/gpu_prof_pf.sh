#!/bin/bash
# Kernel trace of a short bench run + per-dispatch PMC summary (VALU / wait / LDS counters) of every
# kernel, for each pyramid+FAST path in PATHS (default: fused legacy).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for path in ${PATHS:-fused legacy}; do
  D=gpurun_out/pf_$path
  mkdir -p $D
  CMD="python bench.py --steps 3 --warmup 1 --stage-steps 1 --no-cpu-baseline --no-parity --matcher-steps 0 --rectify-steps 0 --no-side-configs --path $path ${BENCH_ARGS}"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- $CMD > $D/trace.log 2>&1 || { tail -20 $D/trace.log; exit 1; }
  echo "=== $path"
  python tools/pf_trace_summary.py $D/trace
  i=0
  for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $D/p$i -o run -- $CMD > $D/p$i.log 2>&1 || { tail -20 $D/p$i.log; exit 1; }
  done
  python tools/pf_pmc_summary.py $D
done
