#!/bin/bash
# GPU: the round's committed counter set for the default bench workload, on the isolated-timing
# build (variants/liborbfe_iso.so = -DFAST_NO_OVERLAP: every launch in stream order, so each
# kernel's trace duration is its own): kernel trace + issue / wave-state, HBM traffic (FETCH_SIZE,
# WRITE_SIZE) and cache / LDS counters, one rocprofv3 --pmc pass per group.
# Summarise with: python tools/pmc_round.py gpurun_out/prof_round <prefix>
set -o pipefail
cd $GRAFT_REPO_ROOT
export ORBFE_LIB_PARTIAL=1   # A/B baselines built from older commits may predate entry points
export TMPDIR=/tmp
D=gpurun_out/prof_round
mkdir -p $D
LIB=$PWD/${ISO_LIB:-variants/liborbfe_iso.so}
PCMD="python bench.py --frames 512 --steps 3 --warmup 1 --stage-steps 1 --no-cpu-baseline --no-parity --matcher-steps 0 --rectify-steps 2 --no-side-configs"
ORBFE_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- $PCMD > $D/trace.log 2>&1 || { tail -20 $D/trace.log; exit 1; }
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  ORBFE_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $D/p$i -o run -- $PCMD > $D/p$i.log 2>&1 || { tail -20 $D/p$i.log; exit 1; }
done
python tools/pmc_round.py $D ${PREFIX:-rXX} --outdir gpurun_out --images 1024
