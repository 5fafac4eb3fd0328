"""Per-level work counters of k_pyrfast (a -DPF_STATS build): one 512-image 752x480 batch."""
import ctypes
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from orb_slam3_ros_amd import _lib
from orb_slam3_ros_amd.synth import synth_stereo
lib = _lib.load(sys.argv[1])
lib.orbfe_debug_pf_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
dev = torch.device("cuda", 0)
W, H, B = 752, 480, 512
pairs = [synth_stereo(i, W, H) for i in range(8)]
imgs = torch.from_numpy(np.stack([pairs[i % 8][i % 2] for i in range(B)])).to(dev)
h = ctypes.c_void_p()
lib.orbfe_extractor_create(1000, 1.2, 8, 20, 7, ctypes.byref(h))
ptrs = (ctypes.c_void_p * B)(*[imgs[i].data_ptr() for i in range(B)])
st = np.zeros(64, np.uint64)
lib.orbfe_debug_pf_stats(st.ctypes.data, 1)
lib.orbfe_extract_batch(h, B, ptrs, W, H, W, 0, 0, None)
lib.orbfe_debug_pf_stats(st.ctypes.data, 1)
names = ["groups", "entries", "corners", "wave-blocks", "chunks", "surv", "fallback", "bands"]
for l in range(8):
    print(l, {n: int(st[8 * l + i]) for i, n in enumerate(names)})
