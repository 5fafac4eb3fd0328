# GPU: full parity suite, bench line, rocprofv3 kernel stats, PMC FETCH/WRITE passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -3 gpurun_out/tests.log
timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --matcher-steps 0 ${BENCH_ARGS} > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
CMD="python bench.py --steps 2 --warmup 1 --stage-steps 1 --no-cpu-baseline --matcher-steps 0 ${BENCH_ARGS}"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- $CMD > gpurun_out/pmc/p$i.log 2>&1 || { tail -20 gpurun_out/pmc/p$i.log; exit 1; }
done
find gpurun_out/prof gpurun_out/pmc -name "*.csv" | head -20
mkdir -p gpurun_out/pmcc
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmcc/c$i -o run -- $CMD > gpurun_out/pmcc/c$i.log 2>&1 || { tail -20 gpurun_out/pmcc/c$i.log; exit 1; }
done
