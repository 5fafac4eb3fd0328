"""GPU probe: two-camera last-frame searches (k_sbp_block2) on synthetic frames, per case the device
time (HIP events), passes, Hamming pairs and the wall time of the host call.
usage: python tools/block2_probe.py"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros_amd import synth_match as sm  # noqa: E402
from orb_slam3_ros_amd.matcher import ORBmatcher  # noqa: E402

m = ORBmatcher(0.9, True)
lib = m._lib
for nl, nr, npts, cf, th in [(1000, 1000, 1600, 0.9, 7), (1000, 1000, 1600, 0.9, 14), (1000, 900, 1500, 0.8, 7),
                             (300, 280, 2000, 0.97, 7)]:
    rng = np.random.default_rng(nl + npts)
    F = sm.synth_frame_two(rng, nl, nr, w=512, h=512)
    pts, ruv = sm.synth_proj_points_two(rng, F, npts, copy_frac=cf)
    mvp0, obs = sm.initial_slots(rng, F.N, 0.2)
    for _ in range(3):
        m.SearchByProjectionLastFrameStereo(F, mvp0.copy(), obs, pts, ruv, th, False, False)
    lib.orbfe_matcher_set_stats(1)
    n = m.SearchByProjectionLastFrameStereo(F, mvp0.copy(), obs, pts, ruv, th, False, False)
    lib.orbfe_matcher_set_stats(0)
    st = (ctypes.c_longlong * 3)()
    lib.orbfe_matcher_last_stats(st)
    lib.orbfe_matcher_set_timing(1)
    dev = []
    for _ in range(10):
        m.SearchByProjectionLastFrameStereo(F, mvp0.copy(), obs, pts, ruv, th, False, False)
        dev.append(lib.orbfe_matcher_last_ms())
    lib.orbfe_matcher_set_timing(0)
    bufs = [mvp0.copy() for _ in range(20)]
    t0 = time.perf_counter()
    for b in bufs:
        m.SearchByProjectionLastFrameStereo(F, b, obs, pts, ruv, th, False, False)
    wall = (time.perf_counter() - t0) / 20 * 1e3
    print(f"nl {nl} nr {nr} pts {npts} copy {cf} th {th}: matches {n} passes {st[2]} pairs {st[1]} "
          f"device {np.median(dev):.4f} ms wall {wall:.4f} ms", flush=True)
