#!/bin/bash
# GPU: throughput A/B of variants/liborbfe_*.so (ORBFE_LIB): the default bench workload with the
# post-timing parity check, no CPU / matcher / rectify / side-config legs; REPS rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
for so in variants/liborbfe_*.so; do
  n=$(basename $so .so)
  ORBFE_LIB=$PWD/$so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --matcher-steps 0 --rectify-steps 0 --no-side-configs ${BENCH_ARGS} > gpurun_out/va_$n.json 2> gpurun_out/va_$n.err || { tail -20 gpurun_out/va_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/va_$n.json'));print('$n', d['value'], d['ms_per_step'], d['stage_ms'], d['parity']['ok'])"
done
done
