#!/usr/bin/env python3
"""GPU diagnostic of the drop-in Tracking frame (tests/native/capi_frontend.cpp --tracking-diag): per
matcher call the wall time, the device time (HIP events around its kernels) and the fixed-point
passes, over the bench's seeded stereo sequence."""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from orb_slam3_ros_amd import build as B  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 40
with tempfile.TemporaryDirectory() as d:
    job = bench.write_sequence_job(os.path.join(d, "seq.bin"), frames)
    r = subprocess.run([B.CAPI_BIN, "--tracking-diag", str(frames), job], capture_output=True, text=True, timeout=300)
    print(r.stdout.strip())
    if r.returncode:
        print(r.stderr[-2000:], file=sys.stderr)
        sys.exit(r.returncode)
