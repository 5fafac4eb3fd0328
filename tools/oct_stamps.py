#!/usr/bin/env python3
"""GPU: per-phase s_memtime stamps of k_octree (image 0 of the batch, every level) on the default
bench workload, from a -DORBFE_OCT_STAMPS build (ORBFE_LIB=variants/liborbfe_stamps.so). Prints the
cycles between consecutive stamps per level: gather, initial nodes, then per step (order / sort,
children, key sweep), then retain + output.

usage: ORBFE_LIB=... python tools/oct_stamps.py [--frames 512]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from orb_slam3_ros_amd.frontend import StereoFrontEnd
    from orb_slam3_ros_amd.synth import synth_stereo
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=512)
    a = ap.parse_args()
    W, H, F = 752, 480, a.frames
    pairs = [synth_stereo(i, W, H) for i in range(16)]
    imgs = np.stack([p[k] for i in range(F) for p in [pairs[i % 16]] for k in (0, 1)])
    dev = torch.device("cuda", 0)
    t = torch.from_numpy(imgs).to(dev)
    fe = StereoFrontEnd(F, W, H, device=dev)
    for _ in range(3):
        fe.run(t)
    torch.cuda.synchronize()
    ts = np.zeros(64, np.uint64)
    for l in range(8):
        n = fe.lib.orbfe_debug_copy(fe.h, 4, 0, l, ts.ctypes.data, ts.nbytes)
        if n <= 0:
            print("no stamps (build with -DORBFE_OCT_STAMPS)")
            return 1
        k = int(ts[63])
        d = np.diff(ts[:min(k, 62)].astype(np.int64))
        info = int(ts[62])
        print(f"level {l}: {k} stamps, total {int(ts[min(k, 62) - 1] - ts[0])} cycles: {d.tolist()}"
              f" (last sort m={info & 0xffff} n={(info >> 16) & 0xffff} K={info >> 32})")
    if hasattr(fe.lib, "orbfe_debug_sort_stamps"):
        st = np.zeros(272, np.uint64)
        fe.lib.orbfe_debug_sort_stamps(ctypes.c_void_p(st.ctypes.data))
        t0 = int(st[0])
        for w in range(16):
            k = int(st[w * 16 + 15])
            if k:
                print(f"sort w{w}:", [int(st[w * 16 + j]) - t0 for j in range(1, min(k, 15))])
        k = int(st[256 + 15])
        print("s64 (wave 0, last call):", np.diff(st[256:256 + min(k, 15)].astype(np.int64)).tolist())
    return 0


if __name__ == "__main__":
    sys.exit(main())
