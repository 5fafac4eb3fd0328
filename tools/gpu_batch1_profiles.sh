#!/bin/bash
# GPU: rocprofv3 kernel-trace summaries of the batch-1 paths kept under profiles/: the pinhole drop-in
# frame (capi_frontend --latency), the pinhole Tracking frame (--tracking) and the KannalaBrandt8
# Tracking frame (--tracking-kb8), 60 frames each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/b1prof
mkdir -p $D
python3 tools/dropin_job.py /tmp/job.bin || exit 1
python3 -c "import bench; bench.write_sequence_job('/tmp/seq.bin', 60); bench.write_sequence_job('/tmp/kb8.bin', 60, 512, 512, 1000, 20, 31, (256.0, 256.0))" || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D/lat -o run -- tests/native/capi_frontend --latency 60 /tmp/job.bin > $D/lat.log 2>&1 || { tail -20 $D/lat.log; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trk -o run -- tests/native/capi_frontend --tracking 60 /tmp/seq.bin /tmp/trk.out > $D/trk.log 2>&1 || { tail -20 $D/trk.log; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kb8 -o run -- tests/native/capi_frontend --tracking-kb8 60 /tmp/kb8.bin /tmp/kb8.out > $D/kb8.log 2>&1 || { tail -20 $D/kb8.log; exit 1; }
for n in lat trk kb8; do
  cp $(find $D/$n -name '*kernel_stats.csv' | head -1) $D/${n}_kernel_stats.csv
  echo "== $n"; python3 - $D/${n}_kernel_stats.csv <<'PY'
import csv, sys
for r in list(csv.reader(open(sys.argv[1])))[1:14]:
    print("  ", r[0][:50], r[1], round(float(r[3]) / 1e3, 2), "us")
PY
done
rm -rf $D/lat $D/trk $D/kb8
