#!/bin/bash
# GPU: config-5 parity at N = 5000 on the in-tree library, then bench.matcher_config5_n(.., 5000)
# device times for variants/liborbfe_{base,st2}.so, two alternating runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_matcher.py \
  -k "sbp_local" > gpurun_out/wq_tests.log 2>&1 || { tail -30 gpurun_out/wq_tests.log; exit 1; }
tail -1 gpurun_out/wq_tests.log
for rep in 1 2; do for v in st2 wth2 wth1; do
  ORBFE_LIB_PARTIAL=1 ORBFE_LIB=$PWD/variants/liborbfe_$v.so timeout -k 10 200 python -c "
import bench
r = bench.matcher_config5_n(10, 5000)
print('$v', {k: (v['device_ms_per_call'], v['parity_ok']) for k, v in r['per_th'].items()})" || exit 1
done; done
