set -o pipefail
cd $GRAFT_REPO_ROOT
ORBFE_LIB_PARTIAL=1 ORBFE_LIB=$PWD/variants/liborbfe_bstamps.so timeout -k 10 120 python tools/blk_scale_probe.py > gpurun_out/bst.log 2>&1 || { tail -5 gpurun_out/bst.log; exit 1; }
grep -v "^blk" gpurun_out/bst.log; for q in 50 800 2000; do grep "nq $q " gpurun_out/bst.log | tail -2; done
