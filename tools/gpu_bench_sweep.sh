# GPU: bench sweep over pipeline counts / batch sizes (no tests).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for args in "--pipelines 1" "--pipelines 2" "--pipelines 4" "--pipelines 2 --frames 512" "--pipelines 4 --frames 512"; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $args > gpurun_out/sweep.json 2> gpurun_out/sweep.err || { tail -20 gpurun_out/sweep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sweep.json'));print('$args', d['value'], d['ms_per_step'])"
done
