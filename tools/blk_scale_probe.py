"""GPU probe: k_sbp_block<1> device time against the number of last-frame points (1000-keypoint
frame, th 7): does the one-workgroup search scale with its queries (LDS / issue contention) or is it
a fixed chain? usage: python tools/blk_scale_probe.py"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros_amd import synth_match as sm  # noqa: E402
from orb_slam3_ros_amd.matcher import ORBmatcher  # noqa: E402

m = ORBmatcher(0.9, True)
lib = m._lib
rng = np.random.default_rng(4242)
F = sm.synth_frame(rng, 1000)
mvp0, obs = sm.initial_slots(rng, F.N, 0.1)
for nq in (50, 100, 200, 400, 800, 1200, 1600, 2000):
    pts = sm.synth_proj_points(np.random.default_rng(nq), F, nq)
    for _ in range(3):
        m.SearchByProjectionLastFrame(F, mvp0.copy(), obs, pts, 7, False, False)
    lib.orbfe_matcher_set_stats(1)
    n = m.SearchByProjectionLastFrame(F, mvp0.copy(), obs, pts, 7, False, False)
    lib.orbfe_matcher_set_stats(0)
    st = (ctypes.c_longlong * 3)()
    lib.orbfe_matcher_last_stats(st)
    lib.orbfe_matcher_set_timing(1)
    dev = []
    for _ in range(15):
        m.SearchByProjectionLastFrame(F, mvp0.copy(), obs, pts, 7, False, False)
        dev.append(lib.orbfe_matcher_last_ms())
    lib.orbfe_matcher_set_timing(0)
    print(f"nq {nq:5d}: matches {n:4d} passes {st[2]:3d} pairs {st[1]:6d} device {np.median(dev) * 1e3:7.1f} us", flush=True)
