#!/bin/bash
# GPU: config-5 matcher device time per th for every variants/liborbfe_*.so (tools/matcher_ab.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export ORBFE_LIB_PARTIAL=1   # A/B baselines built from older commits may predate entry points
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-2}); do
for so in variants/liborbfe_*.so; do
  echo -n "$(basename $so .so) "
  ORBFE_LIB=$PWD/$so timeout -k 10 200 python tools/matcher_ab.py ${CALLS:-30} 2>/dev/null | tail -1 || exit 1
done
done
