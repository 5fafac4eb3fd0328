#!/bin/bash
# GPU: counters of the config-5 search kernels per th (k_sbp_multi0 + k_sbp_multi below th 4,
# k_sbp_band above; one rocprofv3 --pmc pass per counter group), summarised into
# gpurun_out/${PREFIX}_pmc_matcher.json by tools/matcher_pmc_summary.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for th in 1 3 5 15; do
  i=0
  for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAVES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"; do
    i=$((i+1))
    D=gpurun_out/mp_th${th}_$i
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_sbp_(local|band|multi)" --kernel-trace --output-format csv -d $D -o run -- python tools/matcher_run.py $th 20 > $D.log 2>&1 || { tail -20 $D.log; exit 1; }
  done
done
python tools/matcher_pmc_summary.py gpurun_out ${PREFIX:-r05}
