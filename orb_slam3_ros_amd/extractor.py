"""ORBextractor — host mirror of ORB_SLAM3::ORBextractor (include/ORBextractor.h:43-112) over the
C-ABI. Same constructor arguments, getters, operator() semantics (returns monoIndex, -1 on an
empty image; mask ignored; vLappingArea reorders keypoints with x in [lap0, lap1] to the back,
ORBextractor.cc:1153-1162) and a lazily materialised mvImagePyramid.

All compute runs in the HIP kernels of liborbfe.so; this file only moves buffers.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KEYPOINT_DTYPE.itemsize == 28


class ORBextractor:
    HARRIS_SCORE = 0
    FAST_SCORE = 1

    def __init__(self, nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int, minThFAST: int):
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(self._lib.orbfe_extractor_create(int(nfeatures), float(scaleFactor), int(nlevels),
                                                    int(iniThFAST), int(minThFAST), ctypes.byref(h)),
                   "orbfe_extractor_create")
        self._h = h
        self.nfeatures, self.nlevels = int(nfeatures), int(nlevels)
        self._scale_factor = float(np.float32(scaleFactor))
        n = self.nlevels
        self._tabs = {k: np.zeros(n, np.float32) for k in ("scale", "inv", "s2", "inv_s2")}
        self._per_level = np.zeros(n, np.int32)
        _lib.check(self._lib.orbfe_extractor_scale_info(
            h, self._tabs["scale"].ctypes.data, self._tabs["inv"].ctypes.data, self._tabs["s2"].ctypes.data,
            self._tabs["inv_s2"].ctypes.data, self._per_level.ctypes.data), "scale_info")
        self._last_shape = None

    # ---- getters (ORBextractor.h:61-81) ----
    def GetLevels(self) -> int:
        return _lib.check(self._lib.orbfe_extractor_levels(self._h), "orbfe_extractor_levels")

    def GetScaleFactor(self) -> float:
        return self._scale_factor

    def GetScaleFactors(self) -> list[float]:
        return [float(v) for v in self._tabs["scale"]]

    def GetInverseScaleFactors(self) -> list[float]:
        return [float(v) for v in self._tabs["inv"]]

    def GetScaleSigmaSquares(self) -> list[float]:
        return [float(v) for v in self._tabs["s2"]]

    def GetInverseScaleSigmaSquares(self) -> list[float]:
        return [float(v) for v in self._tabs["inv_s2"]]

    @property
    def features_per_level(self) -> list[int]:
        return [int(v) for v in self._per_level]

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def set_opencv_model(self, resize_simd_lanes: int = 16, blur_variant: int = 0):
        """Select the OpenCV build behaviour to reproduce (orbfe_extractor_set_opencv_model):
        cv::resize's universal-intrinsic lane count (0, 8, 16, 32, 64) and the GaussianBlur Q8
        kernel (0 = error diffusion, 1 = per-tap rounding)."""
        _lib.check(self._lib.orbfe_extractor_set_opencv_model(self._h, int(resize_simd_lanes), int(blur_variant)),
                   "orbfe_extractor_set_opencv_model")

    def opencv_model(self) -> tuple[int, int]:
        lanes, blur = ctypes.c_int(), ctypes.c_int()
        _lib.check(self._lib.orbfe_extractor_get_opencv_model(self._h, ctypes.byref(lanes), ctypes.byref(blur)),
                   "orbfe_extractor_get_opencv_model")
        return lanes.value, blur.value

    def capacity(self, width: int, height: int) -> int:
        return _lib.check(self._lib.orbfe_extractor_capacity(self._h, int(width), int(height)), "capacity")

    # ---- operator() (ORBextractor.cc:1086-1168) ----
    def __call__(self, image, mask=None, vLappingArea=(0, 0)):
        """Returns (monoIndex, keypoints[structured KEYPOINT_DTYPE], descriptors[n, 32] u8)."""
        img = np.asarray(image)
        if img.size == 0:
            return -1, np.zeros(0, KEYPOINT_DTYPE), np.zeros((0, 32), np.uint8)
        if img.dtype != np.uint8 or img.ndim != 2:
            raise _lib.OrbfeError("ORBextractor expects a single-channel uint8 image (CV_8UC1)")
        img = np.ascontiguousarray(img)
        h, w = img.shape
        cap = self.capacity(w, h)
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = ctypes.c_int()
        rc = self._lib.orbfe_extract(self._h, img.ctypes.data, w, h, w, int(vLappingArea[0]), int(vLappingArea[1]),
                                     kps.ctypes.data, desc.ctypes.data, cap, ctypes.byref(n))
        _lib.check(rc, "orbfe_extract")
        self._last_shape = (h, w)
        return rc, kps[: n.value].copy(), desc[: n.value].copy()

    def pyramid_level(self, level: int, image: int = 0) -> np.ndarray:
        w, h = ctypes.c_int(), ctypes.c_int()
        _lib.check(self._lib.orbfe_pyramid_level(self._h, image, level, None, 0, ctypes.byref(w), ctypes.byref(h)),
                   "pyramid_level")
        out = np.zeros((h.value, w.value), np.uint8)
        _lib.check(self._lib.orbfe_pyramid_level(self._h, image, level, out.ctypes.data, w.value, None, None),
                   "pyramid_level")
        return out

    @property
    def mvImagePyramid(self) -> list[np.ndarray]:
        """Host copy of the last call's pyramid (levels of image 0), as Frame reads it."""
        return [self.pyramid_level(l) for l in range(self.nlevels)]

    def close(self):
        if getattr(self, "_h", None):
            self._lib.orbfe_extractor_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def descriptor_distance(a, b) -> int:
    """ORBmatcher::DescriptorDistance (ORBmatcher.cc:2058-2074)."""
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return _lib.load().orbfe_descriptor_distance(a.ctypes.data, b.ctypes.data)


def compute_stereo_matches(left: ORBextractor, right: ORBextractor, bf: float, fx: float, n_left: int):
    """Frame::ComputeStereoMatches (Frame.cc:811-981) for the last extract() of both extractors.
    Returns (mvuRight, mvDepth, n_matches_before_cut)."""
    ur = np.zeros(max(n_left, 1), np.float32)
    dp = np.zeros(max(n_left, 1), np.float32)
    rc = _lib.load().orbfe_stereo_match(left.handle, right.handle, float(bf), float(fx), ur.ctypes.data,
                                        dp.ctypes.data)
    _lib.check(rc, "orbfe_stereo_match")
    return ur[:n_left], dp[:n_left], rc


def frame_stereo(left: ORBextractor, right: ORBextractor, imLeft, imRight, bf: float, fx: float):
    """Frame::Frame(stereo) (Frame.cc:101-141) in one library call: ExtractORB on both images (the
    reference's two per-frame threads, :122-125) as one two-image batch on `left`, then
    ComputeStereoMatches (:141). Returns ((monoLeft, kpsLeft, descLeft), (monoRight, kpsRight,
    descRight), mvuRight, mvDepth, n_matches_before_cut)."""
    L = np.ascontiguousarray(np.asarray(imLeft))
    R = np.ascontiguousarray(np.asarray(imRight))
    if L.size == 0 or R.size == 0:
        raise _lib.OrbfeError("Frame(stereo) needs two non-empty images")
    for im in (L, R):
        if im.dtype != np.uint8 or im.ndim != 2:
            raise _lib.OrbfeError("ORBextractor expects a single-channel uint8 image (CV_8UC1)")
    if L.shape != R.shape:
        raise _lib.OrbfeError("left and right images differ in size")
    h, w = L.shape
    cap = left.capacity(w, h)
    kl, kr = np.zeros(cap, KEYPOINT_DTYPE), np.zeros(cap, KEYPOINT_DTYPE)
    dl, dr = np.zeros((cap, 32), np.uint8), np.zeros((cap, 32), np.uint8)
    ur, dp = np.zeros(cap, np.float32), np.zeros(cap, np.float32)
    nl, nr, ml, mr = (ctypes.c_int() for _ in range(4))
    rc = _lib.load().orbfe_frame_stereo(left.handle, right.handle, L.ctypes.data, R.ctypes.data, w, h, w,
                                        float(bf), float(fx), kl.ctypes.data, dl.ctypes.data, cap,
                                        ctypes.byref(nl), ctypes.byref(ml), kr.ctypes.data, dr.ctypes.data, cap,
                                        ctypes.byref(nr), ctypes.byref(mr), ur.ctypes.data, dp.ctypes.data)
    _lib.check(rc, "orbfe_frame_stereo")
    left._last_shape = (h, w)
    n, m = nl.value, nr.value
    return ((ml.value, kl[:n].copy(), dl[:n].copy()), (mr.value, kr[:m].copy(), dr[:m].copy()),
            ur[:n].copy(), dp[:n].copy(), rc)


def frame_fisheye(left: ORBextractor, right: ORBextractor, imLeft, imRight, lap=(0, 511), ratio: float = 0.7):
    """Frame::Frame(stereo, KannalaBrandt8) (Frame.cc:1034-1105) up to the descriptor stage in one library
    call: ExtractORB on both images with vLappingArea `lap` (:1059-1062) as one two-image batch on `left`,
    then ComputeStereoFishEyeMatches' knnMatch(k=2) + ratio over the lapping rows (:1126-1151).
    Returns ((monoLeft, kpsLeft, descLeft), (monoRight, kpsRight, descRight), l2r, dist, n_good):
    l2r[i] = the right keypoint index of left keypoint i whose ratio test passes, else -1."""
    L = np.ascontiguousarray(np.asarray(imLeft))
    R = np.ascontiguousarray(np.asarray(imRight))
    if L.size == 0 or R.size == 0:
        raise _lib.OrbfeError("Frame(stereo) needs two non-empty images")
    for im in (L, R):
        if im.dtype != np.uint8 or im.ndim != 2:
            raise _lib.OrbfeError("ORBextractor expects a single-channel uint8 image (CV_8UC1)")
    if L.shape != R.shape:
        raise _lib.OrbfeError("left and right images differ in size")
    h, w = L.shape
    cap = left.capacity(w, h)
    kl, kr = np.zeros(cap, KEYPOINT_DTYPE), np.zeros(cap, KEYPOINT_DTYPE)
    dl, dr = np.zeros((cap, 32), np.uint8), np.zeros((cap, 32), np.uint8)
    l2r, dist = np.zeros(cap, np.int32), np.zeros(cap, np.int32)
    nl, nr, ml, mr = (ctypes.c_int() for _ in range(4))
    rc = _lib.load().orbfe_frame_fisheye(left.handle, right.handle, L.ctypes.data, R.ctypes.data, w, h, w,
                                         int(lap[0]), int(lap[1]), float(ratio), kl.ctypes.data, dl.ctypes.data, cap,
                                         ctypes.byref(nl), ctypes.byref(ml), kr.ctypes.data, dr.ctypes.data, cap,
                                         ctypes.byref(nr), ctypes.byref(mr), l2r.ctypes.data, dist.ctypes.data)
    _lib.check(rc, "orbfe_frame_fisheye")
    left._last_shape = (h, w)
    n, m = nl.value, nr.value
    return ((ml.value, kl[:n].copy(), dl[:n].copy()), (mr.value, kr[:m].copy(), dr[:m].copy()), l2r[:n].copy(),
            dist[:n].copy(), rc)

