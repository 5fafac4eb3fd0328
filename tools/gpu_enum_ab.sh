#!/bin/bash
# GPU: the pinhole and KB8 Tracking harnesses (tests/native/capi_frontend --tracking / --tracking-kb8,
# 60-frame seeded sequences) with every variants_lat/<name>/liborbfe.so, 3 alternating runs, each
# run's per-frame slots compared with the CPU twin's (tests/native/tracking_cpu).
set -o pipefail
cd $GRAFT_REPO_ROOT
D=/tmp/enum_ab
mkdir -p $D
python3 -c "import bench; bench.write_sequence_job('$D/seq.bin', 60); bench.write_sequence_job('$D/kb8.bin', 60, 512, 512, 1000, 20, 31, (256.0, 256.0))" || exit 1
timeout -k 10 300 tests/native/tracking_cpu 60 $D/seq.bin $D/cpu.out > /dev/null || exit 1
timeout -k 10 300 tests/native/tracking_cpu --kb8 60 $D/kb8.bin $D/cpu_kb8.out > /dev/null || exit 1
for r in 1 2 3; do
  for d in variants_lat/*/; do
    n=$(basename $d)
    LD_LIBRARY_PATH=$PWD/$d:$LD_LIBRARY_PATH timeout -k 10 120 tests/native/capi_frontend --tracking 60 $D/seq.bin $D/g.out > $D/t.json || exit 1
    a=$(cmp -s $D/g.out $D/cpu.out && echo ok || echo MISMATCH)
    LD_LIBRARY_PATH=$PWD/$d:$LD_LIBRARY_PATH timeout -k 10 120 tests/native/capi_frontend --tracking-kb8 60 $D/kb8.bin $D/gk.out > $D/k.json || exit 1
    b=$(cmp -s $D/gk.out $D/cpu_kb8.out && echo ok || echo MISMATCH)
    python3 -c "
import json, sys
t = json.loads(open('$D/t.json').read().strip().splitlines()[-1]); k = json.loads(open('$D/k.json').read().strip().splitlines()[-1])
print('$n', 'pinhole', t['tracking_frame_ms'], t['split_ms'], '$a', '| kb8', k['tracking_frame_ms'], k['split_ms'], '$b')"
  done
done
# the host-API calls (bench.matcher_calls) with each variant
for r in 1 2; do for d in variants_lat/*/; do
  ORBFE_LIB_PARTIAL=1 ORBFE_LIB=$PWD/$d/liborbfe.so timeout -k 10 120 python3 -c "
import bench
r = bench.matcher_calls(20)['calls']
print('$(basename $d)', {k[:24]: (v['ms_per_call'], v['device_ms_per_call'], v['parity_ok']) for k, v in r.items()})" || exit 1
done; done
