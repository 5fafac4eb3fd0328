#!/bin/bash
# GPU: k_sbp_band's skip of unchanged queries: local-map parity tests, then config-5 kernel traces
# (th 5 / 15, 30 device-resident calls) of variants/liborbfe_{base,skip}.so, two alternating runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_matcher.py \
  -k "sbp_local or search_local" > gpurun_out/band_tests.log 2>&1 || { tail -30 gpurun_out/band_tests.log; exit 1; }
tail -2 gpurun_out/band_tests.log
for rep in 1 2; do
for v in base skip; do
for th in 5 15; do
  D=gpurun_out/bs_${v}_${th}_$rep
  ORBFE_LIB=$PWD/variants/liborbfe_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/config5_trace.py $th 30 > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
  python3 - $D $v $th <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.reader(open(f)))[1:]
tot = sum(float(r[2]) for r in rows if "k_sbp_band" in r[0])
cnt = sum(int(r[1]) for r in rows if "k_sbp_band" in r[0])
print(f"{sys.argv[2]:5s} th {sys.argv[3]:>2s}: k_sbp_band {cnt} launches, {tot / 1e3 / 30:.1f} us per call")
allk = sum(float(r[2]) for r in rows if not r[0].startswith("__amd"))
cw = [float(r[3]) / 1e3 for r in rows if "k_mt_commit_write" in r[0]]
print(f"      all kernels {allk / 1e3 / 30:.1f} us per call; k_mt_commit_write mean {cw[0] if cw else 0:.2f} us")
PY
done; done; done
