# GPU: bench value with 1 / 2 / 4 pipelines (sub-batches on separate HIP streams), two alternating runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do for p in 1 2 4; do
  timeout -k 10 200 python bench.py --pipelines $p --steps 20 --warmup 5 --no-cpu-baseline --matcher-steps 0 --dropin-frames 0 --rectify-steps 0 --no-side-configs --parity-frames 16 > gpurun_out/pl_$p.json 2> gpurun_out/pl_$p.err || { tail -20 gpurun_out/pl_$p.err; exit 1; }
  echo "pipelines $p: $(python tools/show_bench.py gpurun_out/pl_$p.json value ms_per_step)"
done; done
