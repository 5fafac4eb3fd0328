"""Tracking-sized single-camera searches through the host C-ABI (k_sbp_block's workloads): 800
last-frame points (th 7) and 1700 local-map points (th 1) against a 1000-keypoint stereo frame,
`calls` times each, for kernel traces of A/B builds: python tools/blk_probe.py [calls]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np

from orb_slam3_ros_amd import synth_match as sm
from orb_slam3_ros_amd.matcher import ORBmatcher

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 30
rng = np.random.default_rng(777)
F = sm.synth_frame(rng, 1000)
pts = sm.synth_proj_points(rng, F, 800)
mps = sm.synth_local_map(rng, F, 1700, copy_frac=0.6)
mvp0, obs = sm.initial_slots(rng, F.N, 0.1)
m = ORBmatcher(0.9, True)
ml = ORBmatcher(0.8)
for _ in range(calls):
    n1 = m.SearchByProjectionLastFrame(F, mvp0.copy(), obs, pts, 7, False, False)
    n2 = ml.SearchByProjectionLocalMap(F, mvp0.copy(), obs, mps, 1.0)
print("lastframe", n1, "local", n2)
