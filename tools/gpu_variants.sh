# GPU: bench each variants/liborbfe_*.so (ORBFE_LIB override) - kernel A/B experiments.
set -o pipefail
cd $GRAFT_REPO_ROOT
for so in variants/liborbfe_*.so; do
  ORBFE_LIB=$PWD/$so timeout -k 10 200 python bench.py --steps 10 --warmup 3 --stage-steps 5 --no-cpu-baseline --matcher-steps 0 --rectify-steps 0 ${BENCH_ARGS} > gpurun_out/var.json 2> gpurun_out/var.err || { tail -20 gpurun_out/var.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/var.json'));print(sys.argv[1], d['value'], d['stage_ms'])" $so
done
