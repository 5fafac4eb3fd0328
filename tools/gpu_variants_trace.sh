#!/bin/bash
# GPU: kernel-trace each variants/liborbfe_*.so (ORBFE_LIB override) on a short bench run and print
# per-kernel mean durations (kernel A/B experiments; ablated variants produce invalid outputs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export ORBFE_LIB_PARTIAL=1   # A/B baselines built from older commits may predate entry points
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-2}); do
for so in variants/liborbfe_*.so; do
  n=$(basename $so .so)
  D=gpurun_out/vt_${n}_$rep
  mkdir -p $D
  ORBFE_LIB=$PWD/$so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python bench.py --steps 5 --warmup 2 --stage-steps 1 --no-cpu-baseline --no-parity --matcher-steps 0 --rectify-steps 0 --no-side-configs ${BENCH_ARGS} > $D/log 2>&1 || { tail -20 $D/log; exit 1; }
  echo "=== $n $(grep -o '"value": [0-9.]*' $D/log | head -1)"
  python tools/trace_grid_summary.py $D | grep -v "k_copy"
done
done
