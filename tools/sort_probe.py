#!/usr/bin/env python3
"""GPU: calls orbfe_debug_block_sort (k_debug_block_sort, one 256-thread block) on octree-like
expandable-node arrays ((size << 44) | (x0 << 32) | position, many ties) of several lengths, REPS
times each, in order; run under rocprofv3 --kernel-trace and pair the trace rows with the sizes
printed here (tools/gpu_sort_probe.sh).

usage: ORBFE_LIB=... python tools/sort_probe.py [reps]
"""
import ctypes
import os
import sys

import numpy as np

SIZES = (40, 120, 300, 600, 1200, 2400)


def make(n, rng):
    size = rng.integers(2, 9, n).astype(np.uint64)
    x0 = rng.integers(0, 48, n).astype(np.uint64) * 16
    return (size << np.uint64(44)) | (x0 << np.uint64(32)) | np.arange(n, dtype=np.uint64)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    lib = ctypes.CDLL(os.environ.get("ORBFE_LIB", os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "orb_slam3_ros_amd", "liborbfe.so")))
    lib.orbfe_debug_block_sort.argtypes = [ctypes.c_void_p, ctypes.c_int]
    rng = np.random.default_rng(7)
    for n in SIZES:
        for _ in range(reps):
            a = make(n, rng)
            assert lib.orbfe_debug_block_sort(a.ctypes.data, n) == n
    print("sizes", " ".join(map(str, SIZES)), "reps", reps)


if __name__ == "__main__":
    main()
