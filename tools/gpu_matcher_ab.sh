#!/bin/bash
# GPU: config-5 matcher leg (host, device and resident times per th) for each variants/liborbfe_*.so.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
for so in variants/liborbfe_*.so; do
  n=$(basename $so .so)
  ORBFE_LIB=$PWD/$so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --stage-steps 0 --no-cpu-baseline --no-parity --rectify-steps 0 --no-side-configs --matcher-steps 40 > gpurun_out/mt_$n.json 2> gpurun_out/mt_$n.err || { tail -20 gpurun_out/mt_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/mt_$n.json'))['matcher_config5']['per_th'];print('$n', {k:(v['device_ms_per_call'],v['resident_ms_per_call'],v['nmatches']) for k,v in d.items() if k.startswith('th')})"
done
done
