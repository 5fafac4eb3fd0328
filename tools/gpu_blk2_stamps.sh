# GPU: phase stamps of k_sbp_block2 (variants/stampdir/liborbfe.so, -DORBFE_BLK2_STAMPS) on the
# synthetic probe and the KB8 Tracking harness.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ORBFE_LIB_PARTIAL=1 ORBFE_LIB=$PWD/variants/stampdir/liborbfe.so timeout -k 10 120 python tools/block2_probe.py > gpurun_out/b2probe.log 2>&1 || { tail -20 gpurun_out/b2probe.log; exit 1; }
grep -v "^blk2" gpurun_out/b2probe.log; grep "^blk2" gpurun_out/b2probe.log | tail -4
python -c "import bench; bench.write_sequence_job('/tmp/kb8.bin', 60, 512, 512, 1000, 20, 31, (256.0, 256.0))"
LD_LIBRARY_PATH=$PWD/variants/stampdir timeout -k 10 120 tests/native/capi_frontend --tracking-kb8 60 /tmp/kb8.bin /tmp/kb8.out > gpurun_out/kb8s.json 2> gpurun_out/kb8s.err || { tail -20 gpurun_out/kb8s.err; exit 1; }
grep "^blk2" gpurun_out/kb8s.json | tail -8; grep -c "^blk2" gpurun_out/kb8s.json
