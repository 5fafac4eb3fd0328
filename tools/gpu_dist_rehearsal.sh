# GPU box: 2 ranks on cuda:0 over gloo (rehearsal of the multi-rank bench path incl. the slab exchange).
# Plain `bench.py --gpus 2`: bench.py spawns its own torchrun child.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --gpus 2 --steps 4 --warmup 2 --frames 64 --dist-backend gloo --same-device --no-cpu-baseline --matcher-steps 0 --rectify-steps 0 --stage-steps 1 > gpurun_out/dist.json 2> gpurun_out/dist.err || { tail -30 gpurun_out/dist.err; exit 1; }
python tools/show_bench.py gpurun_out/dist.json n_gpus value config config4_multi_gpu config4_multi_gpu_k1
