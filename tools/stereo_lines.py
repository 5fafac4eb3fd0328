"""CPU estimate of k_stereo's compulsory HBM traffic: the distinct 128-byte lines that the SAD
refinement windows of Frame::ComputeStereoMatches (Frame.cc:900-930: an 11x11 left window and an
11x21 right window per left keypoint that reaches it) touch in the two images' level buffers, laid
out as the extractor lays them out (level 0 = the caller's image, pitch W; levels 1.. packed with a
64-byte-rounded pitch). Uses the oracle's keypoints and uR (uR0 ~ round(uR): within a pixel, which
moves a window by at most one line edge). usage: python tools/stereo_lines.py [pairs]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402
from orb_slam3_ros_amd.synth import synth_stereo  # noqa: E402

oracle.build()
BF, FX = 0.110078 * 458.654, 458.654
pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
W, H = 752, 480
sf = 1.2 ** np.arange(8)
tot_lines, tot_kp, tot_req = 0, 0, 0
for s in range(pairs):
    L, R = synth_stereo(100 + s, W, H)
    ol, orr = oracle.OracleExtractor(1000, 1.2, 8, 20, 7), oracle.OracleExtractor(1000, 1.2, 8, 20, 7)
    ml, kl, dl = ol(L)
    mr, kr, dr = orr(R)
    ur, dp, nm = oracle.stereo_match(ol, orr, kl, dl, kr, dr, BF, FX)
    ol.close()
    orr.close()
    lines = set()
    req = 0
    for i in np.nonzero(ur >= 0)[0]:
        lv = int(kl["octave"][i])
        inv = 1.0 / sf[lv]
        w_l = int(round(W * inv)) if lv else W
        pitch = W if lv == 0 else ((int(np.ceil(W / sf[lv])) + 63) // 64) * 64
        uL, vL = round(float(kl["x"][i]) * inv), round(float(kl["y"][i]) * inv)
        uR0 = round(float(ur[i]) * inv)
        r0, c0L, c0R = int(vL - 5), int(uL - 5), int(uR0 - 10)
        for side, c0, wdt in ((0, c0L, 11), (1, c0R, 21)):
            for y in range(r0, r0 + 11):
                a0 = (side, lv, (y * pitch + c0) // 128)
                a1 = (side, lv, (y * pitch + c0 + wdt + 3) // 128)   # the kernel's dword over-read
                lines.add(a0)
                lines.add(a1)
                req += 1 + (a1 != a0)
    tot_lines += len(lines)
    tot_kp += int((ur >= 0).sum())
    tot_req += req
print(f"{pairs} pairs: {tot_kp / pairs:.0f} refined keypoints per frame, {tot_req / pairs:.0f} line requests, "
      f"{tot_lines / pairs:.0f} distinct lines = {tot_lines * 128 / pairs / 1e6:.3f} MB per frame; "
      f"line reuse {1 - tot_lines / tot_req:.2f}")
