"""Print the octree's per-phase s_memtime stamps (image 0, every level) for one synthetic batch."""
import ctypes, os, sys
os.environ["ORBFE_OCT_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from orb_slam3_ros_amd.frontend import StereoFrontEnd
from orb_slam3_ros_amd.synth import synth_stereo
F = int(sys.argv[1]) if len(sys.argv) > 1 else 256
l, r = synth_stereo(1)
host = np.stack([l, r] * F)
imgs = torch.from_numpy(host).cuda()
fe = StereoFrontEnd(F, 752, 480)
for _ in range(3):
    fe.run(imgs)
torch.cuda.synchronize()
for lv in range(8):
    ts = np.zeros(64, np.uint64)
    fe.lib.orbfe_debug_copy(fe.h, 4, 0, lv, ts.ctypes.data, ts.nbytes)
    n = int(ts[63])
    t = ts[:min(n, 62)].astype(np.int64)
    print("level", lv, "stamps", n, "deltas(cycles):", (t[1:] - t[:-1]).tolist(), "total", int(t[-1] - t[0]))
