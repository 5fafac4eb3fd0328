# GPU: per-dispatch PMC counters of one bench step (one counter group per rocprofv3 run), summarised
# per dispatch (kernel, duration, counters) by tools/pmc_dispatch_summary.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcd
export TMPDIR=/tmp
CMD="python bench.py --steps 1 --warmup 1 --stage-steps 0 --no-cpu-baseline --matcher-steps 0 --rectify-steps 0 ${BENCH_ARGS}"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT" \
           "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmcd/p$i -o run -- $CMD > gpurun_out/pmcd/p$i.log 2>&1 || { tail -20 gpurun_out/pmcd/p$i.log; echo "pass $i failed"; }
done
python tools/pmc_dispatch_summary.py gpurun_out/pmcd
