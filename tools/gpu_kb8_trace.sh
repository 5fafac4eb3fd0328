# GPU: kernel trace of the KB8 Tracking harness (tests/native/capi_frontend --tracking-kb8, 60 frames).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import bench; bench.write_sequence_job('/tmp/kb8.bin', 60, 512, 512, 1000, 20, 31, (256.0, 256.0))"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kb8prof -o run -- tests/native/capi_frontend --tracking-kb8 60 /tmp/kb8.bin /tmp/kb8.out > gpurun_out/kb8prof.log 2>&1 || { tail -20 gpurun_out/kb8prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/kb8prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.reader(open(f)))[1:16]:
    print("  ", r[0][:50], r[1], round(float(r[3]) / 1e3, 2), "us")
PY
