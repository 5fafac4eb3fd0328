"""Write the job file of the batch-1 drop-in latency run (bench.py dropin_leg's input):
python tools/dropin_job.py OUT.bin [W H NFEATURES]"""
import os
import struct
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from orb_slam3_ros_amd.synth import synth_stereo

out = sys.argv[1]
W, H, nf = (int(a) for a in (sys.argv[2:5] if len(sys.argv) >= 5 else (752, 480, 1000)))
left, right = synth_stereo(7, W, H)
with open(out, "wb") as f:
    f.write(struct.pack("<5i2f", W, H, nf, 0, 100, 0.110078 * 458.654, 458.654) + left.tobytes() + right.tobytes())
