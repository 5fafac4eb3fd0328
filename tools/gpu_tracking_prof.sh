# GPU: kernel trace of the pinhole Tracking harness (tests/native/capi_frontend --tracking, 60 frames).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import bench; bench.write_sequence_job('/tmp/seq.bin', 60)"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trkprof -o run -- tests/native/capi_frontend --tracking 60 /tmp/seq.bin /tmp/trk.out > gpurun_out/trkprof.log 2>&1 || { tail -20 gpurun_out/trkprof.log; exit 1; }
tail -c 600 gpurun_out/trkprof.log
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/trkprof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.reader(open(f)))[1:16]:
    print("  ", r[0][:50], r[1], round(float(r[3]) / 1e3, 2), "us")
PY
