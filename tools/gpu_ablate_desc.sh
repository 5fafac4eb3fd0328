set -o pipefail
cd $GRAFT_REPO_ROOT
for m in 0 1 2 3; do
  ORBFE_ABLATE_DESC=$m ORBFE_LIB=${ORBFE_LIB:-} timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --matcher-steps 0 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('ablate $m', d['stage_ms'])"
done
