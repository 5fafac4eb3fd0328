"""Config-5 SearchByProjection(local map) calls at one th through the host C-ABI (the workload of
bench.py's matcher_config5), for a rocprofv3 counter pass: python tools/matcher_run.py TH CALLS"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np

from orb_slam3_ros_amd import synth_match as sm
from orb_slam3_ros_amd.matcher import ORBmatcher

th, calls = float(sys.argv[1]), int(sys.argv[2])
rng = np.random.default_rng(12345)
F = sm.synth_frame(rng, 1000)
mps = sm.synth_local_map(rng, F, 100_000)
mvp0, obs = sm.initial_slots(rng, F.N)
m = ORBmatcher(0.8)
for _ in range(calls):
    n = m.SearchByProjectionLocalMap(F, mvp0.copy(), obs, mps, th)
print("th", th, "nmatches", n)
