"""Batched device front-end: extract(L) + extract(R) + the stereo matcher for many stereo frames
per launch sequence (the multi-frame / multi-camera path of BASELINE config 2-4).

Frame f of a batch is images (2f, 2f+1) of one interleaved [2F, H, W] u8 device tensor: this is
the batched form of Frame::Frame(stereo) (Frame.cc:101-197), which runs ORBextractor::operator()
on the left and right image on two threads (Frame.cc:122-125) and then ComputeStereoMatches
(Frame.cc:141, :811-981). Outputs are device tensors in the reference's order (mvKeys,
mDescriptors, mvuRight, mvDepth per frame, padded to `cap`).

stereo="fisheye" is the KannalaBrandt8 constructor (Frame.cc:1007-1075): each side is extracted
with its camera's vLappingArea (Frame.cc:1059-1060) and ComputeStereoFishEyeMatches' descriptor
stage (knnMatch k=2 over the lapping rows + Lowe's 0.7, Frame.cc:1126-1151) runs batched on the
device; `l2r` holds the mvLeftToRightMatch candidates the host-side TriangulateMatches filters.

torch is used only for device memory and streams; all compute is in liborbfe.so.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .extractor import KEYPOINT_DTYPE


class StereoFrontEnd:
    """`pipelines` > 1 splits the frames into that many sub-batches, each with its own engine handle
    and HIP stream, so the kernels of different sub-batches overlap on the GPU (the latency-bound
    octree / stereo stages of one sub-batch run beside the streaming stages of another)."""

    def __init__(self, frames: int, width: int, height: int, nfeatures: int = 1000, scale_factor: float = 1.2,
                 nlevels: int = 8, ini_th: int = 20, min_th: int = 7, bf: float = 0.110078 * 458.654,
                 fx: float = 458.654, device=None, pipelines: int = 1, lap_left=(0, 0), lap_right=(0, 0),
                 stereo: str = "rectified", knn_ratio: float = 0.7):
        import torch
        self.torch = torch
        self.lib = _lib.load()
        self.F, self.W, self.H = int(frames), int(width), int(height)
        self.bf, self.fx = float(bf), float(fx)
        if stereo not in ("rectified", "fisheye", "none"):
            raise ValueError(f"stereo must be 'rectified', 'fisheye' or 'none', not {stereo!r}")
        self.stereo, self.knn_ratio = stereo, float(knn_ratio)
        self.lap_left = (int(lap_left[0]), int(lap_left[1]))
        self.lap_right = (int(lap_right[0]), int(lap_right[1]))
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        P = max(1, min(int(pipelines), self.F))
        bounds = [self.F * i // P for i in range(P + 1)]
        self.parts = [(bounds[i], bounds[i + 1]) for i in range(P) if bounds[i + 1] > bounds[i]]
        self.handles, self.streams = [], []
        for _ in self.parts:
            h = ctypes.c_void_p()
            _lib.check(self.lib.orbfe_extractor_create(nfeatures, scale_factor, nlevels, ini_th, min_th,
                                                       ctypes.byref(h)), "create")
            self.handles.append(h)
            # an explicit stream per pipeline: the library's NULL-stream default is its own
            # non-blocking stream, which torch's default stream would not be ordered against
            self.streams.append(torch.cuda.Stream(self.device))
        self.h = self.handles[0]
        self.cap = _lib.check(self.lib.orbfe_extractor_capacity(self.h, self.W, self.H), "capacity")
        for h in self.handles[1:]:
            self.lib.orbfe_extractor_capacity(h, self.W, self.H)
        n = 2 * self.F
        t = torch
        self.kps = t.zeros((n, self.cap, 7), dtype=t.int32, device=self.device)        # cv::KeyPoint records
        self.desc = t.zeros((n, self.cap, 32), dtype=t.uint8, device=self.device)
        self.counts = t.zeros((n, 2), dtype=t.int32, device=self.device)
        self.uright = t.zeros((self.F, self.cap), dtype=t.float32, device=self.device)
        self.depth = t.zeros((self.F, self.cap), dtype=t.float32, device=self.device)
        self.nmatch = t.zeros((self.F,), dtype=t.int32, device=self.device)
        if stereo == "fisheye":   # mvLeftToRightMatch candidates + their distances
            self.l2r = t.full((self.F, self.cap), -1, dtype=t.int32, device=self.device)
            self.l2r_dist = t.full((self.F, self.cap), -1, dtype=t.int32, device=self.device)
        self.bind_outputs(self.counts, self.kps, self.desc)
        self._ptrs = None
        self._ptr_key = None
        self._stage_on = False
        self._stereo_ev = []

    def bind_outputs(self, counts, kps, desc):
        """Direct the batch outputs (counts [2F,2] i32, keypoints [2F,cap,7] i32, descriptors
        [2F,cap,32] u8, contiguous device tensors) into caller-owned buffers, e.g. the views of a
        distributed.SlabExchange slab; takes effect from the next run()."""
        n, t = 2 * self.F, self.torch
        assert counts.shape == (n, 2) and counts.dtype == t.int32 and counts.is_contiguous()
        assert kps.shape == (n, self.cap, 7) and kps.dtype == t.int32 and kps.is_contiguous()
        assert desc.shape == (n, self.cap, 32) and desc.dtype == t.uint8 and desc.is_contiguous()
        self.counts, self.kps, self.desc = counts, kps, desc
        for h, (a, b) in zip(self.handles, self.parts):
            _lib.check(self.lib.orbfe_set_batch_outputs(h, kps[2 * a].data_ptr(), desc[2 * a].data_ptr(),
                                                        counts[2 * a].data_ptr(), 2 * (b - a)),
                       "set_batch_outputs")

    def _pointer_arrays(self, images):
        key = (images.data_ptr(), tuple(images.shape), tuple(images.stride()))
        if key != self._ptr_key:
            base, st = images.data_ptr(), images.stride(0)
            self._ptrs = [(ctypes.c_void_p * (2 * (b - a)))(*[base + i * st for i in range(2 * a, 2 * b)])
                          for a, b in self.parts]
            self._ptr_key = key
        return self._ptrs

    def run(self, images, stream=None):
        """images: [2F, H, W] uint8 CUDA tensor, contiguous rows (left = even, right = odd).
        stream=None: the work runs on the front end's own torch streams, ordered after and before
        the caller's current stream; otherwise everything is enqueued on `stream` (a hipStream_t)."""
        torch = self.torch
        assert images.dtype == torch.uint8 and images.dim() == 3 and images.is_cuda
        n = images.shape[0]
        assert n == 2 * self.F and images.shape[1] == self.H and images.shape[2] == self.W
        assert images.stride(2) == 1 and images.stride(1) >= self.W
        main = torch.cuda.current_stream(self.device)
        ptrs = self._pointer_arrays(images)
        if stream is None:   # ordered after / before the caller's current torch stream
            ev0 = torch.cuda.Event()
            ev0.record(main)
        for i, (h, st, p, (a, b)) in enumerate(zip(self.handles, self.streams, ptrs, self.parts)):
            if stream is None:
                st.wait_event(ev0)
                s = st.cuda_stream
            else:
                s = stream
            if self.lap_left == self.lap_right:
                _lib.check(self.lib.orbfe_extract_batch(h, 2 * (b - a), p, self.W, self.H, images.stride(1),
                                                        self.lap_left[0], self.lap_left[1], s), "extract_batch")
            else:
                _lib.check(self.lib.orbfe_extract_batch_laps(h, 2 * (b - a), p, self.W, self.H, images.stride(1),
                                                             self._laps(b - a).ctypes.data, s), "extract_batch_laps")
            if self.stereo == "none":
                continue
            timed = self._stage_on and i == 0 and stream is None
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
            if self.stereo == "fisheye":
                _lib.check(self.lib.orbfe_stereo_knn_batch(h, 0, 2, h, 1, 2, b - a, self.knn_ratio,
                                                           self.l2r[a].data_ptr(), self.l2r_dist[a].data_ptr(),
                                                           self.nmatch[a:].data_ptr(), s), "stereo_knn_batch")
            else:
                _lib.check(self.lib.orbfe_stereo_match_batch(h, 0, 2, h, 1, 2, b - a, self.bf, self.fx,
                                                             self.uright[a].data_ptr(), self.depth[a].data_ptr(),
                                                             self.nmatch[a:].data_ptr(), s), "stereo_match_batch")
            if timed:
                e1.record(st)
                self._stereo_ev.append((e0, e1))
        if stream is None:
            for st in self.streams:
                main.wait_stream(st)

    def _laps(self, nframes):
        key = ("laps", nframes)
        if getattr(self, "_lap_key", None) != key:
            self._lap_arr = np.array([*self.lap_left, *self.lap_right] * nframes, np.int32)
            self._lap_key = key
        return self._lap_arr

    def set_opencv_model(self, resize_simd_lanes: int = 16, blur_variant: int = 0):
        """orbfe_extractor_set_opencv_model on every pipeline handle (see ORBextractor.set_opencv_model);
        the handles rebuild their buffers, so the outputs are re-bound."""
        for h in self.handles:
            _lib.check(self.lib.orbfe_extractor_set_opencv_model(h, int(resize_simd_lanes), int(blur_variant)),
                       "set_opencv_model")
            self.lib.orbfe_extractor_capacity(h, self.W, self.H)
        self.bind_outputs(self.counts, self.kps, self.desc)

    def set_stage_timing(self, on: bool):
        for h in self.handles:
            self.lib.orbfe_set_stage_timing(h, 1 if on else 0)
        self._stage_on = bool(on)
        self._stereo_ev = []

    def stage_timing(self):
        """Mean per-batch stage times of the first pipeline (its own stream); "stereo" =
        ComputeStereoMatches (k_stereo + k_stereo_cut), HIP events on the launch stream."""
        ms = np.zeros(_lib.ORBFE_NUM_STAGES, np.float32)
        n = self.lib.orbfe_get_stage_timing(self.handles[0], ms.ctypes.data)
        for h in self.handles[1:]:
            self.lib.orbfe_get_stage_timing(h, np.zeros(_lib.ORBFE_NUM_STAGES, np.float32).ctypes.data)
        out = dict(zip(_lib.STAGE_NAMES, ms.tolist()))
        if self._stereo_ev:
            self.torch.cuda.synchronize(self.device)
            out["stereo"] = float(np.mean([a.elapsed_time(b) for a, b in self._stereo_ev]))
        return out, n

    def host_image(self, i: int):
        """(monoIndex, keypoints (structured), descriptors) of batch image i, copied to the host."""
        n, mono = (int(v) for v in self.counts[i].cpu().numpy())
        kp = self.kps[i, :n].cpu().numpy().view(KEYPOINT_DTYPE).reshape(n)
        return mono, kp, self.desc[i, :n].cpu().numpy()

    def host_frame(self, f: int):
        """(kps_left structured, desc_left, uright, depth) of frame f, copied to the host."""
        _, kp, d = self.host_image(2 * f)
        n = len(kp)
        return kp, d, self.uright[f, :n].cpu().numpy(), self.depth[f, :n].cpu().numpy()

    def close(self):
        for h in self.handles:
            if h:
                self.lib.orbfe_extractor_destroy(h)
        self.handles = []
        self.h = None
