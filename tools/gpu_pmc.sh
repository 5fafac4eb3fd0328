# GPU: PMC counter passes (one counter group per rocprofv3 run, kernel-trace only).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
CMD="python bench.py --steps 2 --warmup 1 --stage-steps 1 --no-cpu-baseline --matcher-steps 0 ${BENCH_ARGS}"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- $CMD > gpurun_out/pmc/p$i.log 2>&1 || { tail -20 gpurun_out/pmc/p$i.log; exit 1; }
done
ls -R gpurun_out/pmc | head -40
