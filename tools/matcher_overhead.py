"""Host-side cost breakdown of the device-resident SearchByProjection call (config 5, th=1 and 3):
wall per call through the Python wrapper, through ctypes directly, and of the Python-side checks."""
import ctypes
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time

import numpy as np
import torch

from orb_slam3_ros_amd import _lib
from orb_slam3_ros_amd import synth_match as sm
from orb_slam3_ros_amd.matcher import DeviceMatchFrame, MAP_POINT_DTYPE, search_by_projection_local_device

rng = np.random.default_rng(12345)
F = sm.synth_frame(rng, 1000)
mps = sm.synth_local_map(rng, F, 100_000)
mvp0, obs = sm.initial_slots(rng, F.N)
dev = torch.device("cuda", 0)
Fd = DeviceMatchFrame(F, dev)
obs_t = torch.from_numpy(obs.copy()).to(dev)
mps_t = torch.from_numpy(mps.view(np.uint8).reshape(-1).copy()).to(dev)
lib = _lib.load()
N = 200
for th in (1.0, 3.0):
    bufs = [torch.from_numpy(mvp0.copy()).to(dev) for _ in range(N + 5)]
    for b in bufs[:5]:
        search_by_projection_local_device(Fd, b, obs_t, mps_t, th)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in bufs[5:]:
        search_by_projection_local_device(Fd, b, obs_t, mps_t, th)
    torch.cuda.synchronize()
    wrap = (time.perf_counter() - t0) / N
    st = torch.cuda.current_stream(dev).cuda_stream
    n = len(mps)
    ptrs = [(b.data_ptr()) for b in bufs[5:]]
    for b in bufs[5:]:
        b.copy_(torch.from_numpy(mvp0))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for p in ptrs:
        lib.orbfe_search_by_projection_local_device(Fd.ref(), p, obs_t.data_ptr(), mps_t.data_ptr(), n, th, 0, 50.0, 0.8, st)
    torch.cuda.synchronize()
    raw = (time.perf_counter() - t0) / N
    lib.orbfe_matcher_set_timing(1)
    dl = []
    for b in bufs[5:50]:
        b.copy_(torch.from_numpy(mvp0))
        search_by_projection_local_device(Fd, b, obs_t, mps_t, th)
        dl.append(lib.orbfe_matcher_last_ms())
    dms = float(np.mean(dl[5:]))
    lib.orbfe_matcher_set_timing(0)
    print({"th": th, "wrapper_ms": round(wrap * 1e3, 4), "ctypes_ms": round(raw * 1e3, 4),
           "device_ms": round(dms, 4), "ctypes_over_device": round(raw * 1e3 / dms, 3)}, flush=True)
