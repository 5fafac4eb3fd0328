"""Time the pyramid+FAST stage of a 512-image 752x480 batch with every library in argv (A/B)."""
import ctypes
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from orb_slam3_ros_amd import _lib
from orb_slam3_ros_amd.synth import synth_stereo

dev = torch.device("cuda", 0)
W, H, B = 752, 480, 512
pairs = [synth_stereo(i, W, H) for i in range(8)]
host = np.stack([pairs[i % 8][i % 2] for i in range(B)])
imgs = torch.from_numpy(host).to(dev)
for path, mode in [(p, m) for p in sys.argv[1:] for m in (0, 1)]:
    lib = _lib.load(path)
    h = ctypes.c_void_p()
    lib.orbfe_extractor_create(1000, 1.2, 8, 20, 7, ctypes.byref(h))
    lib.orbfe_extractor_set_path(h, mode)
    ptrs = (ctypes.c_void_p * B)(*[imgs[i].data_ptr() for i in range(B)])
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        lib.orbfe_extract_batch(h, B, ptrs, W, H, W, 0, 0, s)
    lib.orbfe_set_stage_timing(h, 1)
    for _ in range(10):
        lib.orbfe_extract_batch(h, B, ptrs, W, H, W, 0, 0, s)
    torch.cuda.synchronize()
    ms = np.zeros(3, np.float32)
    lib.orbfe_get_stage_timing(h, ms.ctypes.data)
    print(f"{path:40s} path {mode} pyramid_fast {ms[0]:.4f} ms  octree {ms[1]:.4f}  describe {ms[2]:.4f}", flush=True)
    lib.orbfe_extractor_destroy(h)
