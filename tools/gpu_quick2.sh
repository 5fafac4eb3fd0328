# GPU: extractor parity, quick bench (stage times), octree phase stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_extractor.py tests/test_gpu_sort.py -x -q > gpurun_out/tq.log 2>&1 || { tail -30 gpurun_out/tq.log; exit 1; }
tail -2 gpurun_out/tq.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --matcher-steps 0 --rectify-steps 0 ${BENCH_ARGS} > gpurun_out/bq.json 2> gpurun_out/bq.err || { tail -30 gpurun_out/bq.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bq.json'));print(d['value'],d['ms_per_step'],d['stage_ms'],d['roofline']['frac'])"
if [ -n "$OCT" ]; then timeout -k 10 120 python tools/oct_stamps.py 256 2>&1 | tail -8; fi
