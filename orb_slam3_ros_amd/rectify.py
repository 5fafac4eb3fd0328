"""Stereo rectification before extraction (System::TrackStereo, System.cc:233-240):
cv::remap(im, out, M1, M2, cv::INTER_LINEAR) with the CV_32F maps of
cv::initUndistortRectifyMap (Settings.cc:506-509), on the GPU through liborbfe.so.
`rectify_maps` builds such maps for a pinhole + radial-tangential camera (synthetic calibrations;
the real ones come from the settings YAML)."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib


def remap_linear(src: np.ndarray, mapx: np.ndarray, mapy: np.ndarray) -> np.ndarray:
    """Host convenience: one u8 image, float32 maps of the output size."""
    lib = _lib.load()
    src = np.ascontiguousarray(src, np.uint8)
    mapx = np.ascontiguousarray(mapx, np.float32)
    mapy = np.ascontiguousarray(mapy, np.float32)
    if mapx.shape != mapy.shape or mapx.ndim != 2:
        raise ValueError("maps must be two equal 2-D float32 arrays")
    dh, dw = mapx.shape
    out = np.zeros((dh, dw), np.uint8)
    _lib.check(lib.orbfe_remap_linear(src.ctypes.data, src.shape[1], src.shape[0], src.strides[0], mapx.ctypes.data,
                                      mapy.ctypes.data, dw, dh, out.ctypes.data, out.strides[0]), "remap_linear")
    return out


def remap_linear_batch(src, mapx, mapy, out, stream=None):
    """Device path: src [n, sh, sw] u8 and out [n, dh, dw] u8 CUDA tensors, maps [dh, dw] float32
    CUDA tensors shared by all images. stream: hipStream_t (default: torch's current stream)."""
    import torch
    lib = _lib.load()
    n = src.shape[0]
    if stream is None:   # enqueue on the caller's current torch stream
        stream = torch.cuda.current_stream(src.device).cuda_stream
    if src.stride(2) != 1 or out.stride(2) != 1 or not mapx.is_contiguous() or not mapy.is_contiguous():
        raise ValueError("remap_linear_batch needs row-contiguous images and contiguous maps")
    # per-image base pointers by arithmetic (one data_ptr() per tensor, not per image)
    idx = np.arange(n, dtype=np.uint64)
    src_ptrs = np.uint64(src.data_ptr()) + idx * np.uint64(src.stride(0) * src.element_size())
    dst_ptrs = np.uint64(out.data_ptr()) + idx * np.uint64(out.stride(0) * out.element_size())
    ps = src_ptrs.ctypes.data_as(ctypes.POINTER(ctypes.c_void_p))
    pd = dst_ptrs.ctypes.data_as(ctypes.POINTER(ctypes.c_void_p))
    _lib.check(lib.orbfe_remap_linear_batch(ps, src.shape[2], src.shape[1], src.stride(1), mapx.data_ptr(),
                                            mapy.data_ptr(), out.shape[2], out.shape[1], pd, out.stride(1), n,
                                            stream), "remap_linear_batch")
    return out


def rectify_maps(w: int, h: int, fx: float, fy: float, cx: float, cy: float, dist=(0.0, 0.0, 0.0, 0.0),
                 R=None, P=None):
    """initUndistortRectifyMap(K, D, R, P, (w, h), CV_32F) for k1 k2 p1 p2 (double math, float
    output): for each rectified pixel, the source pixel it samples."""
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], np.float64)
    R = np.eye(3) if R is None else np.asarray(R, np.float64)
    P = K if P is None else np.asarray(P, np.float64)[:3, :3]
    iR = np.linalg.inv(P @ R)
    k1, k2, p1, p2 = dist
    u, v = np.meshgrid(np.arange(w, dtype=np.float64), np.arange(h, dtype=np.float64))
    X = iR[0, 0] * u + iR[0, 1] * v + iR[0, 2]
    Y = iR[1, 0] * u + iR[1, 1] * v + iR[1, 2]
    W = iR[2, 0] * u + iR[2, 1] * v + iR[2, 2]
    x, y = X / W, Y / W
    r2 = x * x + y * y
    kr = 1 + (k1 + k2 * r2) * r2
    xd = x * kr + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * kr + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    return (fx * xd + cx).astype(np.float32), (fy * yd + cy).astype(np.float32)


def undistort_points(pts, K4, dist):
    """cv::undistortPoints(pts, pts, K, D, noArray(), K) of Frame::UndistortKeyPoints on the GPU:
    pts float32 [n, 2], K4 = (fx, fy, cx, cy), dist = 4 / 5 / 8 / 12 OpenCV coefficients."""
    lib = _lib.load()
    p = np.ascontiguousarray(pts, np.float32).reshape(-1, 2)
    k = np.ascontiguousarray(K4, np.float32).reshape(4)
    d = np.ascontiguousarray(dist, np.float32).reshape(-1)
    out = np.zeros_like(p)
    _lib.check(lib.orbfe_undistort_points(p.ctypes.data, len(p), k.ctypes.data, d.ctypes.data, len(d), out.ctypes.data),
               "undistort_points")
    return out
