# GPU: extractor parity tests, then a bench line without the CPU / matcher legs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_extractor.py tests/test_gpu_sort.py -x -q > gpurun_out/tq.log 2>&1 || { tail -30 gpurun_out/tq.log; exit 1; }
tail -2 gpurun_out/tq.log
timeout -k 10 300 python bench.py --no-cpu-baseline --matcher-steps 0 ${BENCH_ARGS} > gpurun_out/bq.json 2> gpurun_out/bq.err || { tail -30 gpurun_out/bq.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bq.json'));print(d['value'],d['ms_per_step'],d['stage_ms'],d['roofline']['frac'])"
