"""Config-5 SearchByProjection calls for a kernel-trace profile (rocprofv3 --kernel-trace --stats)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from orb_slam3_ros_amd import synth_match as sm
from orb_slam3_ros_amd.matcher import DeviceMatchFrame, search_by_projection_local_device

rng = np.random.default_rng(12345)
F = sm.synth_frame(rng, 1000)
mps = sm.synth_local_map(rng, F, 100_000)
mvp0, obs = sm.initial_slots(rng, F.N)
dev = torch.device("cuda", 0)
Fd = DeviceMatchFrame(F, dev)
obs_t = torch.from_numpy(obs.copy()).to(dev)
mps_t = torch.from_numpy(mps.view(np.uint8).reshape(-1).copy()).to(dev)
for th in (1, 15):
    for _ in range(10):
        search_by_projection_local_device(Fd, torch.from_numpy(mvp0.copy()).to(dev), obs_t, mps_t, th)
torch.cuda.synchronize()
print("ok")
