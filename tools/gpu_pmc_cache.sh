# GPU: L2 hit rate and LDS bank-conflict passes (one counter group per rocprofv3 run, kernel-trace only).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcc
export TMPDIR=/tmp
CMD="python bench.py --steps 2 --warmup 1 --stage-steps 1 --no-cpu-baseline --matcher-steps 0 --rectify-steps 0 ${BENCH_ARGS}"
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmcc/c$i -o run -- $CMD > gpurun_out/pmcc/c$i.log 2>&1 || { tail -20 gpurun_out/pmcc/c$i.log; exit 1; }
done
find gpurun_out/pmcc -name "*.csv"
