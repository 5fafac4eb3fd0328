"""ORBmatcher — host mirror of the Tracking-thread methods of ORB_SLAM3::ORBmatcher
(include/ORBmatcher.h:38-109, src/ORBmatcher.cc) over the C-ABI of liborbfe.so.

The reference methods take C++ objects (Frame&, KeyFrame*, MapPoint*); here they take flattened
snapshots with the same fields (include/orbfe.h): `MatchFrame` (mvKeysUn, mDescriptors, mvuRight,
image bounds, mvScaleFactors, mbf), MapPoint records (MAP_POINT_DTYPE / PROJ_POINT_DTYPE) and
DBoW2 FeatureVectors (`FeatureVector`). MapPoint* values are int32 handles (-1 = NULL).
Semantics — query order, "already matched" skips, ratio tests, rotation-consistency histogram
and the returned nmatches — are those of the reference; all compute runs in liborbfe.so's HIP
kernels (no CPU fallback).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .extractor import KEYPOINT_DTYPE

# orbfe_map_point (80 B): MapPoint tracking snapshot (MapPoint.h:172-180)
MAP_POINT_DTYPE = np.dtype([("proj_x", "<f4"), ("proj_y", "<f4"), ("proj_xr", "<f4"), ("view_cos", "<f4"),
                            ("depth", "<f4"), ("scale_level", "<i4"), ("flags", "<i4"), ("observations", "<i4"),
                            ("id", "<i4"), ("proj_yr", "<f4"), ("view_cos_r", "<f4"), ("scale_level_r", "<i4"),
                            ("desc", "u1", (32,))])
# orbfe_proj_point (64 B): a projected point of the last frame / a keyframe
PROJ_POINT_DTYPE = np.dtype([("u", "<f4"), ("v", "<f4"), ("invzc", "<f4"), ("octave", "<i4"), ("angle", "<f4"),
                             ("valid", "<i4"), ("observations", "<i4"), ("id", "<i4"), ("desc", "u1", (32,))])
# orbfe_map_point_3d (80 B): MapPoint geometry for the local-map projection (Frame::isInFrustum)
MAP_POINT_3D_DTYPE = np.dtype([("pos", "<f4", (3,)), ("normal", "<f4", (3,)), ("min_dist", "<f4"), ("max_dist", "<f4"),
                               ("flags", "<i4"), ("observations", "<i4"), ("id", "<i4"), ("track_depth", "<f4"),
                               ("desc", "u1", (32,))])
# orbfe_last_point (64 B): a last-frame point for the device-projected motion-model search
LAST_POINT_DTYPE = np.dtype([("pos", "<f4", (3,)), ("octave", "<i4"), ("angle", "<f4"), ("observations", "<i4"),
                             ("id", "<i4"), ("valid", "<i4"), ("desc", "u1", (32,))])
assert MAP_POINT_DTYPE.itemsize == 80 and PROJ_POINT_DTYPE.itemsize == 64 and MAP_POINT_3D_DTYPE.itemsize == 80
assert LAST_POINT_DTYPE.itemsize == 64
MP_IN_VIEW, MP_BAD, MP_SKIP, MP_IN_VIEW_R = 1, 2, 4, 8
TH_HIGH, TH_LOW, HISTO_LENGTH = 100, 50, 30   # ORBmatcher.cc:33-35


class CFrame(ctypes.Structure):
    """struct orbfe_frame"""
    _fields_ = [("n", ctypes.c_int32), ("keys", ctypes.c_void_p), ("desc", ctypes.c_void_p),
                ("uright", ctypes.c_void_p), ("min_x", ctypes.c_float), ("max_x", ctypes.c_float),
                ("min_y", ctypes.c_float), ("max_y", ctypes.c_float), ("nlevels", ctypes.c_int32),
                ("scale_factors", ctypes.c_void_p), ("mbf", ctypes.c_float), ("two_cams", ctypes.c_int32),
                ("nleft", ctypes.c_int32), ("l2r", ctypes.c_void_p), ("r2l", ctypes.c_void_p),
                ("device", ctypes.c_int32)]


class CFeatureVector(ctypes.Structure):
    """struct orbfe_feature_vector"""
    _fields_ = [("n_nodes", ctypes.c_int32), ("node_ids", ctypes.c_void_p), ("offsets", ctypes.c_void_p),
                ("indices", ctypes.c_void_p)]


class Camera(ctypes.Structure):
    """struct orbfe_camera: Frame::mRcw (row-major), mtcw, mOw, pinhole fx fy cx cy,
    mfLogScaleFactor and the viewing-cosine limit (0.5 in Tracking::SearchLocalPoints)."""
    _fields_ = [("Rcw", ctypes.c_float * 9), ("tcw", ctypes.c_float * 3), ("Ow", ctypes.c_float * 3),
                ("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("log_scale_factor", ctypes.c_float), ("view_cos_limit", ctypes.c_float)]

    @staticmethod
    def make(Rcw, tcw, fx, fy, cx, cy, scale_factor=1.2, view_cos_limit=0.5):
        R = np.asarray(Rcw, np.float32).reshape(3, 3)
        t = np.asarray(tcw, np.float32).reshape(3)
        Ow = (-(R.astype(np.float64).T @ t.astype(np.float64))).astype(np.float32)   # mOw = -Rcw^T tcw
        c = Camera()
        c.Rcw[:] = [float(v) for v in R.reshape(-1)]
        c.tcw[:] = [float(v) for v in t]
        c.Ow[:] = [float(v) for v in Ow]
        c.fx, c.fy, c.cx, c.cy = float(fx), float(fy), float(cx), float(cy)
        # Frame::mfLogScaleFactor = log(mfScaleFactor) on the float factor: the C library logf
        libm = ctypes.CDLL("libm.so.6")
        libm.logf.restype = ctypes.c_float
        libm.logf.argtypes = [ctypes.c_float]
        c.log_scale_factor = float(libm.logf(float(np.float32(scale_factor))))
        c.view_cos_limit = float(view_cos_limit)
        return c


SE3, SIM3 = 0, 1


def _logf(x: float) -> float:
    libm = ctypes.CDLL("libm.so.6")
    libm.logf.restype = ctypes.c_float
    libm.logf.argtypes = [ctypes.c_float]
    return float(libm.logf(float(np.float32(x))))


def rotation_to_quaternion(R) -> np.ndarray:
    """Unit quaternion (x, y, z, w) of a rotation matrix (Eigen's Quaternion(Matrix3) branch
    structure, evaluated in double and rounded to float)."""
    m = np.asarray(R, np.float64).reshape(3, 3)
    tr = m[0, 0] + m[1, 1] + m[2, 2]
    if tr > 0:
        t = np.sqrt(tr + 1.0)
        w = 0.5 * t
        t = 0.5 / t
        q = [(m[2, 1] - m[1, 2]) * t, (m[0, 2] - m[2, 0]) * t, (m[1, 0] - m[0, 1]) * t, w]
    else:
        i = 0
        if m[1, 1] > m[0, 0]:
            i = 1
        if m[2, 2] > m[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = np.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
        q = [0.0, 0.0, 0.0, 0.0]
        q[i] = 0.5 * t
        t = 0.5 / t
        q[3] = (m[k, j] - m[j, k]) * t
        q[j] = (m[j, i] + m[i, j]) * t
        q[k] = (m[k, i] + m[i, k]) * t
    q = np.array(q, np.float64)
    return (q / np.linalg.norm(q)).astype(np.float32)


class Pose(ctypes.Structure):
    """struct orbfe_pose: a Sophus SE3f (unit quaternion) or Sim3f (RxSO3 quaternion, scale |q|^2)."""
    _fields_ = [("q", ctypes.c_float * 4), ("t", ctypes.c_float * 3), ("kind", ctypes.c_int32)]

    @staticmethod
    def se3(R, t):
        p = Pose()
        p.q[:] = [float(v) for v in rotation_to_quaternion(R)]
        p.t[:] = [float(v) for v in np.asarray(t, np.float32).reshape(3)]
        p.kind = SE3
        return p

    @staticmethod
    def sim3(R, t, s):
        p = Pose()
        q = rotation_to_quaternion(R).astype(np.float64) * np.sqrt(float(s))
        p.q[:] = [float(v) for v in q.astype(np.float32)]
        p.t[:] = [float(v) for v in np.asarray(t, np.float32).reshape(3)]
        p.kind = SIM3
        return p

    def rotation(self) -> np.ndarray:
        x, y, z, w = [float(v) for v in self.q]
        n = x * x + y * y + z * z + w * w
        x, y, z, w = (v / np.sqrt(n) for v in (x, y, z, w))
        return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                         [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                         [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])

    def scale(self) -> float:
        return float(sum(float(v) ** 2 for v in self.q)) if self.kind == SIM3 else 1.0


class CameraModel(ctypes.Structure):
    """struct orbfe_camera_model: GeometricCamera type + mvParameters (fx fy cx cy [k0 k1 k2 k3])."""
    _fields_ = [("type", ctypes.c_int32), ("params", ctypes.c_float * 8)]

    PINHOLE, KANNALA_BRANDT8 = 0, 1

    @staticmethod
    def make(kind, fx, fy, cx, cy, k=(0.0, 0.0, 0.0, 0.0)):
        m = CameraModel()
        m.type = CameraModel.KANNALA_BRANDT8 if kind in ("kb8", CameraModel.KANNALA_BRANDT8) else CameraModel.PINHOLE
        m.params[:] = [float(np.float32(v)) for v in (fx, fy, cx, cy, *k)]
        return m


class StereoRig(ctypes.Structure):
    """struct orbfe_stereo_rig: Frame::mpCamera / mpCamera2, mTrl (rotation row-major, translation),
    mTlr.translation() and mRwc (row-major), as Frame::isInFrustumChecks reads them (Frame.cc:1168-1242)."""
    _fields_ = [("left", CameraModel), ("right", CameraModel), ("Rrl", ctypes.c_float * 9), ("trl", ctypes.c_float * 3),
                ("tlr", ctypes.c_float * 3), ("Rwc", ctypes.c_float * 9)]

    @staticmethod
    def make(left: CameraModel, right: CameraModel = None, Tlr=None, Rcw=None):
        """Tlr: 4x4 right-to-left transform (Stereo.T_c1_c2); Rcw: the frame rotation (mRwc = Rcw^T)."""
        r = StereoRig()
        r.left = left
        r.right = right if right is not None else left
        T = np.eye(4, dtype=np.float64) if Tlr is None else np.asarray(Tlr, np.float64)
        Rlr, tlr = T[:3, :3], T[:3, 3]
        Rrl = Rlr.T
        trl = -(Rrl @ tlr)
        r.Rrl[:] = [float(v) for v in np.asarray(Rrl, np.float32).reshape(-1)]
        r.trl[:] = [float(v) for v in np.asarray(trl, np.float32)]
        r.tlr[:] = [float(v) for v in np.asarray(tlr, np.float32)]
        R = np.eye(3, dtype=np.float32) if Rcw is None else np.asarray(Rcw, np.float32).reshape(3, 3)
        r.Rwc[:] = [float(v) for v in R.T.reshape(-1)]
        return r


class KFCamera(ctypes.Structure):
    """struct orbfe_kf_camera: the keyframe pose (Sophus), camera centre, pinhole intrinsics and
    mfLogScaleFactor read by the back-end projections."""
    _fields_ = [("Tcw", Pose), ("Ow", ctypes.c_float * 3), ("fx", ctypes.c_float), ("fy", ctypes.c_float),
                ("cx", ctypes.c_float), ("cy", ctypes.c_float), ("log_scale_factor", ctypes.c_float)]

    @staticmethod
    def make(Tcw: Pose, fx, fy, cx, cy, scale_factor=1.2, Ow=None):
        c = KFCamera()
        c.Tcw = Tcw
        if Ow is None:
            R, t = Tcw.rotation(), np.array(Tcw.t[:], np.float64)
            Ow = -(R.T @ t)
        c.Ow[:] = [float(v) for v in np.asarray(Ow, np.float32).reshape(3)]
        c.fx, c.fy, c.cx, c.cy = float(fx), float(fy), float(cx), float(cy)
        c.log_scale_factor = _logf(scale_factor)
        return c


class MatchFrame:
    """The parts of a Frame the matchers read (Frame.h). keys: KEYPOINT_DTYPE [n] (mvKeysUn),
    desc: uint8 [n, 32], bounds: (mnMinX, mnMaxX, mnMinY, mnMaxY), uright: float32 [n] or None.
    Two-camera frame (Nleft != -1): nleft given, keys / desc = mvKeys ++ mvKeysRight, l2r / r2l =
    mvLeftToRightMatch [nleft] / mvRightToLeftMatch [n - nleft] (int32, -1 = none)."""

    def __init__(self, keys, desc, bounds, scale_factors, uright=None, mbf: float = 0.0, nleft=None, l2r=None,
                 r2l=None):
        self.keys = np.ascontiguousarray(keys, KEYPOINT_DTYPE).reshape(-1)
        self.desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        if len(self.keys) != len(self.desc):
            raise ValueError("keys and descriptors differ in length")
        self.uright = None if uright is None else np.ascontiguousarray(uright, np.float32).reshape(-1)
        if self.uright is not None and len(self.uright) != len(self.keys):
            raise ValueError("uright length")
        self.scale_factors = np.ascontiguousarray(scale_factors, np.float32).reshape(-1)
        self.bounds = tuple(float(np.float32(b)) for b in bounds)
        self.mbf = float(mbf)
        self.nleft = None if nleft is None else int(nleft)
        if self.nleft is not None:
            n = len(self.keys)
            if not 0 <= self.nleft <= n:
                raise ValueError("nleft out of range")
            self.l2r = np.ascontiguousarray(np.full(self.nleft, -1) if l2r is None else l2r, np.int32).reshape(-1)
            self.r2l = np.ascontiguousarray(np.full(n - self.nleft, -1) if r2l is None else r2l, np.int32).reshape(-1)
            if len(self.l2r) != self.nleft or len(self.r2l) != n - self.nleft:
                raise ValueError("l2r / r2l lengths must be nleft / n - nleft")
            # an empty side still needs a valid pointer
            self._l2r_buf = self.l2r if len(self.l2r) else np.zeros(1, np.int32)
            self._r2l_buf = self.r2l if len(self.r2l) else np.zeros(1, np.int32)
        self.c = CFrame(len(self.keys), self.keys.ctypes.data, self.desc.ctypes.data,
                        self.uright.ctypes.data if self.uright is not None else None, *self.bounds,
                        len(self.scale_factors), self.scale_factors.ctypes.data, self.mbf,
                        1 if self.nleft is not None else 0, self.nleft or 0,
                        self._l2r_buf.ctypes.data if self.nleft is not None else None,
                        self._r2l_buf.ctypes.data if self.nleft is not None else None)

    @property
    def N(self) -> int:
        return len(self.keys)

    def ref(self):
        return ctypes.byref(self.c)


class FeatureVector:
    """DBoW2::FeatureVector (std::map<NodeId, std::vector<unsigned>>) flattened; node ids ascending."""

    def __init__(self, mapping: dict):
        ids = sorted(int(k) for k in mapping)
        self.node_ids = np.asarray(ids, np.uint32)
        lens = [len(mapping[k]) for k in ids]
        self.offsets = np.zeros(len(ids) + 1, np.int32)
        self.offsets[1:] = np.cumsum(lens, dtype=np.int64)
        self.indices = np.asarray([int(i) for k in ids for i in mapping[k]], np.uint32)
        if self.indices.size == 0:
            self.indices = np.zeros(1, np.uint32)
        self.c = CFeatureVector(len(ids), self.node_ids.ctypes.data, self.offsets.ctypes.data,
                                self.indices.ctypes.data)

    def ref(self):
        return ctypes.byref(self.c)


def _i32(a, n, what):
    a = np.asarray(a)
    if a.dtype != np.int32 or not a.flags.c_contiguous or a.size != n:
        raise ValueError(f"{what} must be a contiguous int32 array of length {n}")
    return a


def _records(a, dtype, what):
    a = np.asarray(a)
    if a.dtype != dtype or not a.flags.c_contiguous:
        raise ValueError(f"{what} must be a contiguous array of dtype {dtype}")
    return a


class ORBmatcher:
    """ORBmatcher(nnratio=0.6, checkOri=true) (ORBmatcher.h:43)."""

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True):
        self._lib = _lib.load()
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)

    @staticmethod
    def DescriptorDistance(a, b) -> int:
        a = np.ascontiguousarray(a, np.uint8)
        b = np.ascontiguousarray(b, np.uint8)
        return int(_lib.load().orbfe_descriptor_distance(a.ctypes.data, b.ctypes.data))

    # SearchByProjection(Frame&, const vector<MapPoint*>&, th=3, bFarPoints=false, thFarPoints=50) (:43-213)
    def SearchByProjectionLocalMap(self, F: MatchFrame, mvp, mvp_obs, map_points, th: float = 3.0,
                                   bFarPoints: bool = False, thFarPoints: float = 50.0) -> int:
        mvp = _i32(mvp, F.N, "mvp")
        mvp_obs = _i32(mvp_obs, F.N, "mvp_obs")
        mps = _records(map_points, MAP_POINT_DTYPE, "map_points")
        return _lib.check(self._lib.orbfe_search_by_projection_local(
            F.ref(), mvp.ctypes.data, mvp_obs.ctypes.data, mps.ctypes.data, len(mps), float(th), int(bFarPoints),
            float(thFarPoints), self.mfNNratio), "SearchByProjection(local map)")

    # SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono) (:1676-1887)
    def SearchByProjectionLastFrame(self, cur: MatchFrame, mvp, mvp_obs, points, th: float, bForward: bool,
                                    bBackward: bool) -> int:
        mvp = _i32(mvp, cur.N, "mvp")
        mvp_obs = _i32(mvp_obs, cur.N, "mvp_obs")
        pts = _records(points, PROJ_POINT_DTYPE, "points")
        return _lib.check(self._lib.orbfe_search_by_projection_lastframe(
            cur.ref(), mvp.ctypes.data, mvp_obs.ctypes.data, pts.ctypes.data, len(pts), float(th), int(bForward),
            int(bBackward), int(self.mbCheckOrientation)), "SearchByProjection(last frame)")

    # the same for a two-camera CurrentFrame (:1794-1858): right_uv float32 [n, 2] = the points
    # projected into the right camera by the caller's camera model
    def SearchByProjectionLastFrameStereo(self, cur: MatchFrame, mvp, mvp_obs, points, right_uv, th: float,
                                          bForward: bool, bBackward: bool) -> int:
        mvp = _i32(mvp, cur.N, "mvp")
        mvp_obs = _i32(mvp_obs, cur.N, "mvp_obs")
        pts = _records(points, PROJ_POINT_DTYPE, "points")
        ruv = np.asarray(right_uv)
        if ruv.dtype != np.float32 or not ruv.flags.c_contiguous or ruv.shape != (len(pts), 2):
            raise ValueError("right_uv must be contiguous float32 [n_points, 2]")
        return _lib.check(self._lib.orbfe_search_by_projection_lastframe_stereo(
            cur.ref(), mvp.ctypes.data, mvp_obs.ctypes.data, pts.ctypes.data, ruv.ctypes.data, len(pts), float(th),
            int(bForward), int(bBackward), int(self.mbCheckOrientation)), "SearchByProjection(last frame, stereo)")

    def SearchByProjectionLastFramePose(self, cur: MatchFrame, mvp, mvp_obs, points, Tcw: "Pose", cam: "CameraModel",
                                        th: float, bForward: bool, bBackward: bool, Trl: "Pose" = None) -> int:
        """SearchByProjection(CurrentFrame, LastFrame, th, bMono) with its projection on the device
        (ORBmatcher.cc:1695-1718, 1794-1796): points = LAST_POINT records (world positions), Tcw =
        CurrentFrame.GetPose(), cam = CurrentFrame.mpCamera, Trl = GetRelativePoseTrl() for a
        two-camera frame."""
        mvp = _i32(mvp, cur.N, "mvp")
        mvp_obs = _i32(mvp_obs, cur.N, "mvp_obs")
        pts = _records(points, LAST_POINT_DTYPE, "points")
        return _lib.check(self._lib.orbfe_search_by_projection_lastframe_pose(
            cur.ref(), mvp.ctypes.data, mvp_obs.ctypes.data, pts.ctypes.data, len(pts), ctypes.byref(Tcw),
            ctypes.byref(Trl) if Trl is not None else None, ctypes.byref(cam), float(th), int(bForward),
            int(bBackward), int(self.mbCheckOrientation)), "SearchByProjection(last frame, device projection)")

    # SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist) (:1889-2010)
    def SearchByProjectionKeyFrame(self, cur: MatchFrame, mvp, points, th: float, ORBdist: int) -> int:
        mvp = _i32(mvp, cur.N, "mvp")
        pts = _records(points, PROJ_POINT_DTYPE, "points")
        return _lib.check(self._lib.orbfe_search_by_projection_kf(
            cur.ref(), mvp.ctypes.data, pts.ctypes.data, len(pts), float(th), int(ORBdist),
            int(self.mbCheckOrientation)), "SearchByProjection(keyframe)")

    def SearchByProjection(self, *args, **kw) -> int:
        """Overload dispatch like the C++ name: (F, mvp, mvp_obs, MAP_POINT records, ...) -> local map;
        (F, mvp, mvp_obs, PROJ_POINT records, th, bForward, bBackward) -> last frame;
        (F, mvp, PROJ_POINT records, th, ORBdist) -> keyframe."""
        if len(args) >= 4 and isinstance(args[3], np.ndarray) and args[3].dtype == MAP_POINT_DTYPE:
            return self.SearchByProjectionLocalMap(*args, **kw)
        if len(args) >= 4 and isinstance(args[3], np.ndarray) and args[3].dtype == PROJ_POINT_DTYPE:
            return self.SearchByProjectionLastFrame(*args, **kw)
        return self.SearchByProjectionKeyFrame(*args, **kw)

    # SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize=10) (:648-763)
    def SearchForInitialization(self, F1: MatchFrame, F2: MatchFrame, vbPrevMatched, vnMatches12,
                                windowSize: int = 10) -> int:
        prev = np.asarray(vbPrevMatched)
        if prev.dtype != np.float32 or not prev.flags.c_contiguous or prev.shape != (F1.N, 2):
            raise ValueError("vbPrevMatched must be contiguous float32 [N1, 2]")
        m12 = _i32(vnMatches12, F1.N, "vnMatches12")
        return _lib.check(self._lib.orbfe_search_for_initialization(
            F1.ref(), F2.ref(), prev.ctypes.data, m12.ctypes.data, int(windowSize), self.mfNNratio,
            int(self.mbCheckOrientation)), "SearchForInitialization")

    # SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& vpMapPointMatches) (:223-425)
    def SearchByBoW(self, kf_keys, kf_desc, kf_map_points, kf_featvec: FeatureVector, F: MatchFrame,
                    f_featvec: FeatureVector):
        """Returns (nmatches, vpMapPointMatches int32 [F.N])."""
        kk = np.ascontiguousarray(kf_keys, KEYPOINT_DTYPE).reshape(-1)
        kd = np.ascontiguousarray(kf_desc, np.uint8).reshape(-1, 32)
        km = _i32(np.ascontiguousarray(kf_map_points, np.int32), len(kk), "kf_map_points")
        out = np.full(F.N, -1, np.int32)
        n = _lib.check(self._lib.orbfe_search_by_bow(
            kk.ctypes.data, kd.ctypes.data, km.ctypes.data, len(kk), kf_featvec.ref(), F.ref(), f_featvec.ref(),
            out.ctypes.data, self.mfNNratio, int(self.mbCheckOrientation)), "SearchByBoW")
        return n, out

    # SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12) (:765-903)
    def SearchByBoWKF(self, keys1, desc1, map_points1, featvec1: FeatureVector, keys2, desc2, map_points2,
                      featvec2: FeatureVector, nleft1: int = -1, nleft2: int = -1):
        """LocalMapping / LoopClosing variant. map_points* = GetMapPointMatches() handles, -1 for
        NULL or bad points; nleft1 / nleft2 = NLeft of a keyframe with a second camera (its right
        indices are skipped, ORBmatcher.cc:800-819), -1 otherwise.
        Returns (nmatches, vpMatches12 int32 [len(keys1)]: KF2 handles or -1)."""
        k1 = np.ascontiguousarray(keys1, KEYPOINT_DTYPE).reshape(-1)
        k2 = np.ascontiguousarray(keys2, KEYPOINT_DTYPE).reshape(-1)
        d1 = np.ascontiguousarray(desc1, np.uint8).reshape(-1, 32)
        d2 = np.ascontiguousarray(desc2, np.uint8).reshape(-1, 32)
        if len(d1) != len(k1) or len(d2) != len(k2):
            raise ValueError("descriptor rows must match the keypoints")
        m1 = _i32(np.ascontiguousarray(map_points1, np.int32), len(k1), "map_points1")
        m2 = _i32(np.ascontiguousarray(map_points2, np.int32), len(k2), "map_points2")
        out = np.full(len(k1), -1, np.int32)
        n = _lib.check(self._lib.orbfe_search_by_bow_kf2(
            k1.ctypes.data, d1.ctypes.data, m1.ctypes.data, len(k1), int(nleft1), featvec1.ref(), k2.ctypes.data,
            d2.ctypes.data, m2.ctypes.data, len(k2), int(nleft2), featvec2.ref(), out.ctypes.data, self.mfNNratio,
            int(self.mbCheckOrientation)), "SearchByBoW(KF, KF)")
        return n, out


    # SearchForTriangulation(pKF1, pKF2, vMatchedPairs, bOnlyStereo, bCoarse) (:907-1146)
    def SearchForTriangulation(self, KF1: MatchFrame, mp1, fv1: FeatureVector, KF2: MatchFrame, mp2,
                               fv2: FeatureVector, F12, ep, level_sigma2_2, bOnlyStereo=False, bCoarse=False):
        """mp1 / mp2: GetMapPoint presence per keypoint (handle or -1). F12 (3x3) and ep (2,) as the
        reference computes them. Returns (nmatches, matches12 int32 [KF1.N]: KF2 index or -1);
        vMatchedPairs = [(i, matches12[i]) for i with matches12[i] >= 0]."""
        m1 = _i32(np.ascontiguousarray(mp1, np.int32), KF1.N, "mp1")
        m2 = _i32(np.ascontiguousarray(mp2, np.int32), KF2.N, "mp2")
        F = np.ascontiguousarray(F12, np.float32).reshape(9)
        e = np.ascontiguousarray(ep, np.float32).reshape(2)
        sg = np.ascontiguousarray(level_sigma2_2, np.float32).reshape(-1)
        if len(sg) < len(KF2.scale_factors):
            raise ValueError("level_sigma2_2 needs one entry per level")
        out = np.full(KF1.N, -1, np.int32)
        n = _lib.check(self._lib.orbfe_search_for_triangulation(
            KF1.ref(), m1.ctypes.data, fv1.ref(), KF2.ref(), m2.ctypes.data, fv2.ref(), F.ctypes.data, e.ctypes.data,
            sg.ctypes.data, int(bOnlyStereo), int(bCoarse), int(self.mbCheckOrientation), out.ctypes.data),
            "SearchForTriangulation")
        return n, out

    # SearchForTriangulation with bCoarse = false and the caller's epipolar test (keyframes with a
    # second camera: KannalaBrandt8::epipolarConstrain on the host, ORBmatcher.cc:1036-1074)
    def SearchForTriangulationEpi(self, KF1: MatchFrame, mp1, fv1: FeatureVector, KF2: MatchFrame, mp2,
                                  fv2: FeatureVector, ep, epipolar, bOnlyStereo=False):
        """epipolar(idx1, idx2) -> bool: pCamera1->epipolarConstrain for that keypoint pair. Returns
        (nmatches, matches12) as SearchForTriangulation. Raises _lib.OrbfeCapacityError when the
        shared vocabulary nodes need more than 16 M candidate slots (orbfe.h): the caller then runs its
        own CPU body for this keyframe pair, as the C++ shim does."""
        m1 = _i32(np.ascontiguousarray(mp1, np.int32), KF1.N, "mp1")
        m2 = _i32(np.ascontiguousarray(mp2, np.int32), KF2.N, "mp2")
        e = np.ascontiguousarray(ep, np.float32).reshape(2)
        out = np.full(KF1.N, -1, np.int32)
        # ctypes swallows an exception raised inside a callback (prints it, returns 0): record the
        # first one and re-raise it after the call, so a failing predicate cannot change the matches
        err = []

        def pred(ctx, i1, i2):
            if err:
                return 0
            try:
                return 1 if epipolar(i1, i2) else 0
            except BaseException as ex:  # noqa: BLE001 - re-raised below
                err.append(ex)
                return 0

        cb = _lib.EPIPOLAR_FN(pred)
        n = _lib.check(self._lib.orbfe_search_for_triangulation_epi(
            KF1.ref(), m1.ctypes.data, fv1.ref(), KF2.ref(), m2.ctypes.data, fv2.ref(), e.ctypes.data,
            int(bOnlyStereo), int(self.mbCheckOrientation), cb, None, out.ctypes.data), "SearchForTriangulation")
        if err:
            raise err[0]
        return n, out

    # Fuse(pKF, vpMapPoints, th) (:1148-1337) / Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (:1339-1455)
    def Fuse(self, KF: MatchFrame, cam: KFCamera, points3d, th=3.0, inv_level_sigma2=None, sim3=False,
             model: "CameraModel" = None, bRight: bool = False):
        """The search half of Fuse: (n_candidates, best_idx, best_dist) per point; the map mutation
        (Replace / AddObservation / vpReplacePoint) is the caller's, in point order. model = the
        keyframe's pCamera (mpCamera, or mpCamera2 with bRight; None = pinhole from cam); bRight
        searches a two-camera keyframe's right grid (ORBmatcher.cc:1148-1298)."""
        pts = _records(points3d, MAP_POINT_3D_DTYPE, "points3d")
        if inv_level_sigma2 is None:
            sf = KF.scale_factors
            inv_level_sigma2 = (np.float32(1.0) / (sf * sf)).astype(np.float32)
        sig = np.ascontiguousarray(inv_level_sigma2, np.float32).reshape(-1)
        if len(sig) < len(KF.scale_factors):
            raise ValueError("inv_level_sigma2 needs one entry per level")
        bi = np.full(len(pts), -1, np.int32)
        bd = np.full(len(pts), -1, np.int32)
        if model is None and not bRight and KF.nleft is None:
            n = self._lib.orbfe_fuse(KF.ref(), ctypes.byref(cam), sig.ctypes.data, pts.ctypes.data, len(pts),
                                     float(th), int(bool(sim3)), bi.ctypes.data, bd.ctypes.data)
        else:
            n = self._lib.orbfe_fuse_rig(KF.ref(), ctypes.byref(cam), ctypes.byref(model) if model is not None else None,
                                         sig.ctypes.data, pts.ctypes.data, len(pts), float(th), int(bool(sim3)),
                                         int(bool(bRight)), bi.ctypes.data, bd.ctypes.data)
        n = _lib.check(n, "Fuse")
        return n, bi, bd

    # SearchByProjection(pKF, Scw, vpPoints, vpMatched, th, ratioHamming) (:427-523) and the
    # vpPointsKFs / vpMatchedKF overload (:525-646)
    def SearchByProjectionSim3(self, KF: MatchFrame, cam: KFCamera, points3d, vpMatched, th=10, ratioHamming=1.0,
                               point_kfs=None, vpMatchedKF=None, model: "CameraModel" = None):
        """vpMatched (and vpMatchedKF with point_kfs) int32 [KF.N] updated in place. model: pKF->mpCamera
        (orbfe_search_by_projection_sim3_rig; None = the pinhole expression on cam). Returns nmatches."""
        pts = _records(points3d, MAP_POINT_3D_DTYPE, "points3d")
        m = _i32(vpMatched, KF.N, "vpMatched")
        pk = mk = None
        if point_kfs is not None:
            pk = _i32(np.ascontiguousarray(point_kfs, np.int32), len(pts), "point_kfs")
            mk = _i32(vpMatchedKF, KF.N, "vpMatchedKF")
        if model is not None:
            return _lib.check(self._lib.orbfe_search_by_projection_sim3_rig(
                KF.ref(), ctypes.byref(cam), ctypes.byref(model), pts.ctypes.data, len(pts),
                None if pk is None else pk.ctypes.data, int(th), float(ratioHamming), m.ctypes.data,
                None if mk is None else mk.ctypes.data), "SearchByProjection(Sim3)")
        return _lib.check(self._lib.orbfe_search_by_projection_sim3(
            KF.ref(), ctypes.byref(cam), pts.ctypes.data, len(pts), None if pk is None else pk.ctypes.data, int(th),
            float(ratioHamming), m.ctypes.data, None if mk is None else mk.ctypes.data), "SearchByProjection(Sim3)")

    # SearchBySim3(pKF1, pKF2, vpMatches12, S12, th) (:1457-1674)
    def SearchBySim3(self, KF1: MatchFrame, KF2: MatchFrame, points1, points2, cam1: KFCamera, cam2: KFCamera,
                     S12: Pose, S21: Pose, th, vpMatches12, matched_idx2=None):
        """points1 / points2: GetMapPointMatches() of each keyframe as MAP_POINT_3D_DTYPE (id -1 = NULL).
        vpMatches12 int32 [KF1.N] updated in place; matched_idx2[i] = KF2 index of the initial match i.
        Returns nFound."""
        p1 = _records(points1, MAP_POINT_3D_DTYPE, "points1")
        p2 = _records(points2, MAP_POINT_3D_DTYPE, "points2")
        if len(p1) != KF1.N or len(p2) != KF2.N:
            raise ValueError("one map-point record per keyframe keypoint")
        m = _i32(vpMatches12, KF1.N, "vpMatches12")
        mi = None if matched_idx2 is None else _i32(np.ascontiguousarray(matched_idx2, np.int32), KF1.N,
                                                    "matched_idx2")
        return _lib.check(self._lib.orbfe_search_by_sim3(
            KF1.ref(), KF2.ref(), p1.ctypes.data, p2.ctypes.data, ctypes.byref(cam1), ctypes.byref(cam2),
            ctypes.byref(S12), ctypes.byref(S21), float(th), m.ctypes.data, None if mi is None else mi.ctypes.data),
            "SearchBySim3")


class DeviceMatchFrame:
    """A MatchFrame whose arrays live in HBM (torch CUDA tensors): the frame argument of the
    *_device entry points. The host struct carries the device pointers."""

    def __init__(self, F: MatchFrame, device):
        import torch
        self.N = F.N
        self.bounds = F.bounds
        self.keys = torch.from_numpy(np.ascontiguousarray(F.keys).view(np.uint8).reshape(-1).copy()).to(device)
        self.desc = torch.from_numpy(F.desc.copy()).to(device)
        self.uright = None if F.uright is None else torch.from_numpy(F.uright.copy()).to(device)
        self.scale_factors = torch.from_numpy(F.scale_factors.copy()).to(device)
        two = getattr(F, "nleft", None) is not None
        if two:   # mvLeftToRightMatch / mvRightToLeftMatch in HBM as well
            self.l2r = torch.from_numpy(F._l2r_buf.copy()).to(device)
            self.r2l = torch.from_numpy(F._r2l_buf.copy()).to(device)
        self.c = CFrame(F.N, self.keys.data_ptr(), self.desc.data_ptr(),
                        self.uright.data_ptr() if self.uright is not None else None, *F.bounds,
                        len(F.scale_factors), self.scale_factors.data_ptr(), F.mbf, 1 if two else 0,
                        F.nleft if two else 0, self.l2r.data_ptr() if two else None,
                        self.r2l.data_ptr() if two else None)

    def ref(self):
        return ctypes.byref(self.c)


def _dev_i32(t, n, what):
    import torch
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.int32 and t.is_contiguous() and
            t.numel() == n):
        raise ValueError(f"{what} must be a contiguous CUDA int32 tensor of length {n}")
    return t


def _dev_records(t, itemsize, what):
    import torch
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.uint8 and t.is_contiguous() and
            t.numel() % itemsize == 0):
        raise ValueError(f"{what} must be a contiguous CUDA uint8 tensor of {itemsize}-byte records")
    return t.numel() // itemsize


def search_by_projection_local_device(F: DeviceMatchFrame, mvp, mvp_obs, mps, th=3.0, bFarPoints=False,
                                      thFarPoints=50.0, nnratio=0.8):
    """SearchByProjection(F, vpMapPoints, th, bFar, thFar) on device-resident data: mvp / mvp_obs
    CUDA int32 [F.N] (mvp updated in place), mps a CUDA uint8 tensor of MAP_POINT_DTYPE records.
    Enqueued after the current torch stream's work. Returns nmatches."""
    import torch
    lib = _lib.load()
    n = _dev_records(mps, MAP_POINT_DTYPE.itemsize, "mps")
    _dev_i32(mvp, F.N, "mvp")
    _dev_i32(mvp_obs, F.N, "mvp_obs")
    st = torch.cuda.current_stream(mvp.device).cuda_stream
    return _lib.check(lib.orbfe_search_by_projection_local_device(
        F.ref(), mvp.data_ptr(), mvp_obs.data_ptr(), mps.data_ptr(), n, float(th), int(bFarPoints),
        float(thFarPoints), float(nnratio), st), "search_by_projection_local_device")


def search_local_points_device(F: DeviceMatchFrame, cam: Camera, points3d, mvp, mvp_obs, th=1.0, bFarPoints=False,
                               thFarPoints=50.0, nnratio=0.8, rig: StereoRig = None):
    """Tracking::SearchLocalPoints on device-resident data (points3d: CUDA uint8 tensor of
    MAP_POINT_3D_DTYPE records). Returns (nmatches, nToMatch)."""
    import torch
    lib = _lib.load()
    n = _dev_records(points3d, MAP_POINT_3D_DTYPE.itemsize, "points3d")
    _dev_i32(mvp, F.N, "mvp")
    _dev_i32(mvp_obs, F.N, "mvp_obs")
    ntm = ctypes.c_int32(0)
    st = torch.cuda.current_stream(mvp.device).cuda_stream
    args = (points3d.data_ptr(), n, mvp.data_ptr(), mvp_obs.data_ptr(), float(th), int(bFarPoints), float(thFarPoints),
            float(nnratio), ctypes.byref(ntm), st)
    if rig is None:
        nm = lib.orbfe_search_local_points_device(F.ref(), ctypes.byref(cam), *args)
    else:
        nm = lib.orbfe_search_local_points_rig_device(F.ref(), ctypes.byref(cam), ctypes.byref(rig), *args)
    nm = _lib.check(nm, "search_local_points_device")
    return nm, int(ntm.value)


def compute_distinctive_descriptors(descriptor_sets):
    """MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:329-403) for many points at once on the
    GPU. descriptor_sets: a list of (N_i, 32) uint8 arrays (the descriptors of each point's
    non-bad observations), or a (desc, offsets) pair of the concatenated rows and N+1 offsets.
    Returns int32 [n_points]: the chosen row of each set, -1 for an empty set."""
    if isinstance(descriptor_sets, tuple):
        desc, offsets = descriptor_sets
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        offsets = np.ascontiguousarray(offsets, np.int32)
    else:
        sets = [np.asarray(d, np.uint8).reshape(-1, 32) for d in descriptor_sets]
        offsets = np.zeros(len(sets) + 1, np.int32)
        offsets[1:] = np.cumsum([len(d) for d in sets])
        desc = np.ascontiguousarray(np.concatenate(sets) if sets else np.zeros((0, 32), np.uint8))
    n = len(offsets) - 1
    if n < 0 or (n >= 0 and offsets[-1] != len(desc)):
        raise ValueError("offsets must end at the number of descriptor rows")
    best = np.full(max(n, 0), -1, np.int32)
    lib = _lib.load()
    _lib.check(lib.orbfe_distinctive_descriptors(desc.ctypes.data, offsets.ctypes.data, n, best.ctypes.data),
               "ComputeDistinctiveDescriptors")
    return best


def is_in_frustum(F: MatchFrame, cam: Camera, points3d, rig: StereoRig = None):
    """Frame::isInFrustum + MapPoint::PredictScale over points3d (MAP_POINT_3D_DTYPE) on the GPU.
    rig (StereoRig): the frame's camera models (KannalaBrandt8 included) and, for a two-camera frame,
    the right view (isInFrustumChecks, Frame.cc:1168-1242); None = pinhole from cam.
    Returns (nToMatch, tracking snapshots as MAP_POINT_DTYPE records)."""
    lib = _lib.load()
    pts = _records(points3d, MAP_POINT_3D_DTYPE, "points3d")
    track = np.zeros(len(pts), MAP_POINT_DTYPE)
    if rig is None:
        n = lib.orbfe_is_in_frustum(F.ref(), ctypes.byref(cam), pts.ctypes.data, len(pts), track.ctypes.data)
    else:
        n = lib.orbfe_is_in_frustum_rig(F.ref(), ctypes.byref(cam), ctypes.byref(rig), pts.ctypes.data, len(pts),
                                        track.ctypes.data)
    return _lib.check(n, "is_in_frustum"), track


def search_local_points(F: MatchFrame, cam: Camera, points3d, mvp, mvp_obs, th: float = 1.0, bFarPoints: bool = False,
                        thFarPoints: float = 50.0, nnratio: float = 0.8, rig: StereoRig = None, track: bool = False):
    """Tracking::SearchLocalPoints' projection + SearchByProjection (Tracking.cc:3404-3453) in one
    device pass (rig: see is_in_frustum). mvp is updated in place. Returns (nmatches, nToMatch), and
    with track=True (nmatches, nToMatch, the isInFrustum records as MAP_POINT_DTYPE): the
    orbfe_search_local_points_track form the C++ shim calls (shim/Tracking_orbfe.cc)."""
    lib = _lib.load()
    pts = _records(points3d, MAP_POINT_3D_DTYPE, "points3d")
    mvp = _i32(mvp, F.N, "mvp")
    mvp_obs = _i32(mvp_obs, F.N, "mvp_obs")
    ntm = ctypes.c_int32(0)
    args = (pts.ctypes.data, len(pts), mvp.ctypes.data, mvp_obs.ctypes.data, float(th), int(bFarPoints),
            float(thFarPoints), float(nnratio), ctypes.byref(ntm))
    if track:
        rec = np.zeros(len(pts), MAP_POINT_DTYPE)
        n = lib.orbfe_search_local_points_track(F.ref(), ctypes.byref(cam), ctypes.byref(rig) if rig is not None else None,
                                                *args, rec.ctypes.data)
        return _lib.check(n, "search_local_points_track"), int(ntm.value), rec
    if rig is None:
        n = lib.orbfe_search_local_points(F.ref(), ctypes.byref(cam), *args)
    else:
        n = lib.orbfe_search_local_points_rig(F.ref(), ctypes.byref(cam), ctypes.byref(rig), *args)
    return _lib.check(n, "search_local_points"), int(ntm.value)


def stereo_knn_ratio(left_desc, right_desc, ratio: float = 0.7):
    """Descriptor stage of Frame::ComputeStereoFishEyeMatches (Frame.cc:1126-1151):
    knnMatch(k=2) + Lowe ratio. Returns (good, train [nl], dist [nl])."""
    lib = _lib.load()
    L = np.ascontiguousarray(left_desc, np.uint8).reshape(-1, 32)
    R = np.ascontiguousarray(right_desc, np.uint8).reshape(-1, 32)
    t = np.full(len(L), -1, np.int32)
    d = np.full(len(L), -1, np.int32)
    g = _lib.check(lib.orbfe_stereo_knn_ratio(L.ctypes.data, len(L), R.ctypes.data, len(R), float(ratio),
                                              t.ctypes.data, d.ctypes.data), "stereo_knn_ratio")
    return g, t, d


def current_frame_view(F: MatchFrame, left, frame_id: int):
    """The device view (orbfe_frame_device_view) of the frame the last orbfe_frame_stereo on extractor
    `left` produced, with F's bounds and mbf: a CFrame whose keys / desc / uR / scale factors are in
    HBM, for the host-API single-camera searches (SearchByProjectionLocalMap / LastFrame /
    search_local_points take it through MatchFrame-compatible `.ref()`). None when stale."""
    c = CFrame()
    ctypes.memmove(ctypes.byref(c), F.ref(), ctypes.sizeof(CFrame))
    if _lib.load().orbfe_frame_device_view(left.handle, int(frame_id), ctypes.byref(c)) != 0:
        return None

    class _View:   # what the search wrappers read of a MatchFrame
        pass
    v = _View()
    v.c, v.N, v.nleft, v.scale_factors, v.bounds, v.keys = c, int(c.n), None, F.scale_factors, F.bounds, F.keys
    v.ref = lambda: ctypes.byref(c)
    return v

