"""GPU diagnostic: the KB8 Tracking sequence's frames (seed 31, 512x512, laps {0, 511}) through
orbfe_frame_fisheye, orbfe_extract x 2 + orbfe_stereo_knn_ratio, and the oracle; per frame, which
outputs differ. usage: python tools/kb8_diag.py [frames]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402
from orb_slam3_ros_amd.extractor import ORBextractor, frame_fisheye  # noqa: E402
from orb_slam3_ros_amd.matcher import stereo_knn_ratio  # noqa: E402
from orb_slam3_ros_amd.synth import synth_stereo_sequence  # noqa: E402

oracle.build()
frames = int(sys.argv[1]) if len(sys.argv) > 1 else 24
lap = (0, 511)
el, er = ORBextractor(1000, 1.2, 8, 20, 7), ORBextractor(1000, 1.2, 8, 20, 7)
e1, e2 = ORBextractor(1000, 1.2, 8, 20, 7), ORBextractor(1000, 1.2, 8, 20, 7)
bad = 0
for k, (L, R) in enumerate(synth_stereo_sequence(31, frames, 512, 512)):
    (ml, kl, dl), (mr, kr, dr), l2r, dist, ng = frame_fisheye(el, er, L, R, lap, 0.7)
    ol, orr = oracle.OracleExtractor(1000, 1.2, 8, 20, 7), oracle.OracleExtractor(1000, 1.2, 8, 20, 7)
    oml, okl, odl = ol(L, lap)
    omr, okr, odr = orr(R, lap)
    ol.close()
    orr.close()
    g, t, d = oracle.stereo_knn_ratio(odl[oml:], odr[omr:], 0.7)
    g2, t2, d2 = stereo_knn_ratio(dl[ml:], dr[mr:], 0.7)
    ml2, kl2, dl2 = e1(L, None, lap)
    mr2, kr2, dr2 = e2(R, None, lap)
    exp = np.full(len(okl), -1, np.int32)
    exp[oml:][t >= 0] = t[t >= 0] + omr
    msg = []
    if (ml, mr) != (oml, omr): msg.append(f"mono {ml},{mr} vs {oml},{omr}")
    if not (np.array_equal(kl.view(np.uint8), okl.view(np.uint8)) and np.array_equal(dl, odl)): msg.append("left kp/desc")
    if not (np.array_equal(kr.view(np.uint8), okr.view(np.uint8)) and np.array_equal(dr, odr)): msg.append("right kp/desc")
    if not (np.array_equal(kl2.view(np.uint8), okl.view(np.uint8)) and np.array_equal(kr2.view(np.uint8), okr.view(np.uint8))):
        msg.append("extract x2 kps")
    if ng != g or not np.array_equal(l2r, exp):
        idx = np.nonzero(l2r != exp)[0][:5]
        msg.append(f"fisheye l2r ({ng} vs {g}) at {idx.tolist()} got {l2r[idx].tolist()} exp {exp[idx].tolist()}")
    if g2 != g or not np.array_equal(t2, t): msg.append(f"knn_ratio ({g2} vs {g})")
    print(k, len(kl), len(kr), ng, "OK" if not msg else "; ".join(msg), flush=True)
    bad += bool(msg)
print("bad frames", bad)
sys.exit(1 if bad else 0)
