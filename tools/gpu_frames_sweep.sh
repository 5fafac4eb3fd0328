set -o pipefail
cd $GRAFT_REPO_ROOT
for fr in 256 512 1024 256 512 1024; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --matcher-steps 0 --rectify-steps 0 --no-side-configs --frames $fr > gpurun_out/fs.json 2> gpurun_out/fs.err || { tail -20 gpurun_out/fs.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/fs.json'));print($fr, d['value'], d['ms_per_step'], d['stage_ms'], d['parity']['ok'])"
done
