# GPU: per-phase instruction counts of k_fast / k_describe: one rocprofv3 --pmc pass per ablation
# mode (ORBFE_ABLATE_FAST / ORBFE_ABLATE_DESC), kernel-trace only
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abpmc
export TMPDIR=/tmp
CMD="python bench.py --steps 2 --warmup 1 --stage-steps 1 --no-cpu-baseline --matcher-steps 0 --rectify-steps 0"
CNT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS"
for m in 0 1 2 3; do
  env_fast=$m; env_desc=$m; [ "$ONLY" = desc ] && env_fast=0; [ "$ONLY" = fast ] && env_desc=0
  ORBFE_ABLATE_FAST=$env_fast ORBFE_ABLATE_DESC=$env_desc timeout -k 10 120 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d gpurun_out/abpmc/m$m -o run -- $CMD > gpurun_out/abpmc/m$m.log 2>&1 || { tail -20 gpurun_out/abpmc/m$m.log; exit 1; }
done
python tools/ablate_pmc_summary.py gpurun_out/abpmc
