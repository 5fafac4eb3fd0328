#!/bin/bash
# k_pyrfast phase ablations (tools/build_variant.sh -DPF_ABL=bits): stage time + VALU / wave cycles.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
timeout -k 10 300 python tools/pf_time.py ${VARIANTS} || exit 1
for v in ${VARIANTS}; do
  n=$(basename $v .so)
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/abl/$n -o run -- python tools/pf_time.py $v > gpurun_out/abl/$n.log 2>&1 || { tail -5 gpurun_out/abl/$n.log; exit 1; }
  echo "== $n"; python tools/pf_pmc_summary.py gpurun_out/abl/$n | grep -A6 "^k_pyrfast" | head -7
done
