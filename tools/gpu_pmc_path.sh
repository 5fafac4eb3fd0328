#!/bin/bash
# GPU: per-kernel instruction / wave-state counters of the bench workload on the isolated-timing
# build (variants/liborbfe_iso.so, -DFAST_NO_OVERLAP) for one pyramid+FAST path (PATH_ARG).
# Summarise with: python tools/pmc_round.py gpurun_out/prof_path <prefix> --outdir gpurun_out
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/prof_path
mkdir -p $D
LIB=$PWD/${ISO_LIB:-variants/liborbfe_iso.so}
PCMD="python bench.py --frames 512 --steps 3 --warmup 1 --stage-steps 1 --no-cpu-baseline --no-parity --matcher-steps 0 --rectify-steps 0 --no-side-configs --path ${PATH_ARG:-stream}"
ORBFE_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- $PCMD > $D/trace.log 2>&1 || { tail -20 $D/trace.log; exit 1; }
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS" \
           ${EXTRA_GRPS}; do
  i=$((i+1))
  ORBFE_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $D/p$i -o run -- $PCMD > $D/p$i.log 2>&1 || { tail -20 $D/p$i.log; exit 1; }
done
python tools/pmc_round.py $D ${PREFIX:-rXX} --outdir gpurun_out --images 1024
