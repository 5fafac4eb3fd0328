"""Device-resident config-5 searches (100k map points, seed 12345) at one th, `calls` times, for kernel
traces: python tools/config5_trace.py TH [calls]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from orb_slam3_ros_amd import synth_match as sm  # noqa: E402
from orb_slam3_ros_amd.matcher import DeviceMatchFrame, search_by_projection_local_device  # noqa: E402

th = float(sys.argv[1])
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rng = np.random.default_rng(12345)
F = sm.synth_frame(rng, 1000)
mps = sm.synth_local_map(rng, F, 100_000)
mvp0, obs = sm.initial_slots(rng, F.N)
dev = torch.device("cuda", 0)
Fd = DeviceMatchFrame(F, dev)
obs_t = torch.from_numpy(obs.copy()).to(dev)
mps_t = torch.from_numpy(mps.view(np.uint8).reshape(-1).copy()).to(dev)
bufs = [torch.from_numpy(mvp0.copy()).to(dev) for _ in range(calls)]
for b in bufs:
    n = search_by_projection_local_device(Fd, b, obs_t, mps_t, th)
torch.cuda.synchronize()
print("th", th, "nmatches", n)
