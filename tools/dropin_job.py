"""Write the sequence job of the batch-1 drop-in latency / Tracking-frame runs (bench.py dropin_leg's
input, tests/native/capi_frontend.cpp SeqJob): python tools/dropin_job.py OUT.bin [FRAMES]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402

bench.write_sequence_job(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 100)
