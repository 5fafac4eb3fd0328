#!/usr/bin/env python3
"""Regenerate the golden fixtures of tests/test_oracle_golden.py.

The reference (ORB-SLAM3 + OpenCV 4.2) cannot be built or run here and ships no fixtures for this
path, so these vectors are produced by the CPU oracle (oracle/orb_oracle.cpp) on seeded synthetic
images. They pin the oracle (and through the GPU parity tests, the HIP kernels) against silent
regressions; their agreement with the real reference is "parity unpinned" (see DESIGN.md).
Model switches used: resize_simd_lanes=16, blur_kernel=0 (error-diffusion).
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle  # noqa: E402
from orb_slam3_ros_amd.synth import synth_image, synth_stereo  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle_golden.npz")


def main():
    oracle.build()
    d = {}
    for name, (w, h, nf, lap, seed) in {
        "euroc_mono": (752, 480, 1000, (0, 1000), 1),
        "euroc_stereo_l": (752, 480, 1200, (0, 0), 2),
        "kitti": (1241, 376, 2000, (0, 0), 3),
        "tumvi": (512, 512, 1000, (0, 511), 4),
    }.items():
        img = synth_image(seed, w, h)
        ex = oracle.OracleExtractor(nf, 1.2, 8, 20, 7)
        mono, kp, desc = ex(img, lap)
        d[name + "_img_sha"] = np.frombuffer(hashlib.sha256(img.tobytes()).digest(), np.uint8)
        d[name + "_kp"] = kp.view(np.uint8).reshape(len(kp), 28)
        d[name + "_desc"] = desc
        d[name + "_mono"] = np.array([mono], np.int32)
        d[name + "_meta"] = np.array([w, h, nf, lap[0], lap[1]], np.int32)
        for l in range(8):
            p = ex.pyramid_level(l)
            d[f"{name}_pyr{l}_sum"] = np.array([int(p.astype(np.int64).sum()), p.shape[0], p.shape[1]], np.int64)
    left, right = synth_stereo(5)
    el, er = oracle.OracleExtractor(1200, 1.2, 8, 20, 7), oracle.OracleExtractor(1200, 1.2, 8, 20, 7)
    _, kl, dl = el(left)
    _, kr, dr = er(right)
    ur, dp, nm = oracle.stereo_match(el, er, kl, dl, kr, dr, 0.110078 * 435.2, 435.2)
    d["stereo_img_sha"] = np.frombuffer(hashlib.sha256(left.tobytes() + right.tobytes()).digest(), np.uint8)
    d["stereo_uright"] = ur
    d["stereo_depth"] = dp
    d["stereo_nmatch"] = np.array([nm], np.int32)
    np.savez_compressed(OUT, **d)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
