"""ctypes wrapper of the CPU ORACLE (oracle/liborb_oracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module. It
is the checker (and the timed CPU baseline), never the product path. Parity status: see the
header of oracle/orb_oracle.cpp ("parity unpinned" w.r.t. the real OpenCV-based reference).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "liborb_oracle.so")
KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])


def build(force: bool = False) -> str:
    srcs = [os.path.join(_HERE, f) for f in ("orb_oracle.cpp", "orb_oracle_match.cpp", "orb_oracle_bow.cpp", "orb_oracle_remap.cpp", "orb_oracle_bench.cpp", "Makefile")]
    if force or not os.path.exists(LIB) or any(os.path.getmtime(s) > os.path.getmtime(LIB) for s in srcs):
        subprocess.run(["make", "-C", _HERE, "-B" if force else "-s"], check=True)
    return LIB


CONTRACT_LIB = os.path.join(_HERE, "liborb_oracle_contract.so")


def build_contract() -> str:
    """The oracle built with the reference's own flags (-O3 -march=native, g++'s default FMA
    contraction; the OpenCV restatements pinned uncontracted): tests/test_oracle_contraction.py."""
    subprocess.run(["make", "-C", _HERE, "-s", "contract"], check=True)
    return CONTRACT_LIB


_lib = None
_libs = {}


def lib(path: str | None = None) -> ctypes.CDLL:
    global _lib
    if path is not None:   # another build of the same sources (the contraction check)
        if path not in _libs:
            _libs[path] = _sigs(ctypes.CDLL(path))
        return _libs[path]
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = _sigs(ctypes.CDLL(LIB))
    return _lib


def _sigs(L: ctypes.CDLL) -> ctypes.CDLL:
    vp, ci, cf = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    L.oro_create.restype = vp
    L.oro_create.argtypes = [ci, cf, ci, ci, ci]
    L.oro_destroy.argtypes = [vp]
    L.oro_set_model.argtypes = [vp, ci, ci]
    L.oro_level_info.argtypes = [vp, vp, vp, vp, vp, vp, vp]
    L.oro_extract.argtypes = [vp, vp, ci, ci, ci, ci, ci, vp, ci, vp, ctypes.POINTER(ci)]
    L.oro_pyramid_level.argtypes = [vp, ci, vp, ci, ctypes.POINTER(ci), ctypes.POINTER(ci)]
    L.oro_debug_keys.argtypes = [vp, ci, ci, vp, ci]
    L.oro_resize.argtypes = [vp, ci, ci, vp, ci, ci, ci]
    L.oro_blur.argtypes = [vp, ci, ci, vp, ci]
    L.oro_fast.argtypes = [vp, ci, ci, ci, ci, vp, ci]
    L.oro_fast_atan2.restype = cf
    L.oro_fast_atan2.argtypes = [cf, cf]
    L.oro_hamming.argtypes = [vp, vp]
    L.oro_stereo_match.argtypes = [vp, vp, vp, vp, ci, vp, vp, ci, cf, cf, vp, vp]
    L.oro_bench_extract.restype = ctypes.c_double
    L.oro_bench_extract.argtypes = [vp, ci, ci, ci, ci, cf, ci, ci, ci, ci, ctypes.POINTER(ci)]
    L.oro_std_sort_u64_hi.argtypes = [vp, ci]
    L.oro_bench_stereo.restype = ctypes.c_long
    L.oro_bench_stereo.argtypes = [vp, vp, ci, ci, ci, ci, cf, ci, ci, ci, cf, cf, ci]
    return L


class OracleExtractor:
    """CPU restatement of ORB_SLAM3::ORBextractor (see oracle/orb_oracle.cpp)."""

    def __init__(self, nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, resize_simd_lanes=16, blur_variant=0,
                 lib_path=None):
        self._l = lib(lib_path)
        self.h = self._l.oro_create(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
        self._l.oro_set_model(self.h, resize_simd_lanes, blur_variant)
        self.nlevels = nlevels

    def level_info(self):
        n = self.nlevels
        out = [np.zeros(n, np.float32) for _ in range(4)] + [np.zeros(n, np.int32), np.zeros(16, np.int32)]
        self._l.oro_level_info(self.h, *[a.ctypes.data for a in out])
        return dict(zip(("scale", "inv_scale", "sigma2", "inv_sigma2", "per_level", "umax"), out))

    def __call__(self, img, lap=(0, 0)):
        img = np.ascontiguousarray(img, np.uint8)
        h, w = img.shape
        cap = 20000
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = ctypes.c_int()
        mono = self._l.oro_extract(self.h, img.ctypes.data, w, h, w, lap[0], lap[1], kps.ctypes.data, cap,
                                   desc.ctypes.data, ctypes.byref(n))
        return mono, kps[: n.value].copy(), desc[: n.value].copy()

    def pyramid_level(self, level):
        w, h = ctypes.c_int(), ctypes.c_int()
        self._l.oro_pyramid_level(self.h, level, None, 0, ctypes.byref(w), ctypes.byref(h))
        out = np.zeros((h.value, w.value), np.uint8)
        self._l.oro_pyramid_level(self.h, level, out.ctypes.data, out.size, ctypes.byref(w), ctypes.byref(h))
        return out

    def debug_keys(self, level, which):
        """which=0: raw FAST keys of the level (vToDistributeKeys, coords relative to minBorder);
        which=1: DistributeOctTree output (level coords, before scaling)."""
        n = self._l.oro_debug_keys(self.h, level, which, None, 0)
        out = np.zeros(n, KEYPOINT_DTYPE)
        self._l.oro_debug_keys(self.h, level, which, out.ctypes.data, n)
        return out

    def close(self):
        if self.h:
            self._l.oro_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def stereo_match(ext_l: OracleExtractor, ext_r: OracleExtractor, kl, dl, kr, dr, bf, fx):
    L = ext_l._l
    n = len(kl)
    ur = np.zeros(max(n, 1), np.float32)
    dp = np.zeros(max(n, 1), np.float32)
    kl = np.ascontiguousarray(kl)
    kr = np.ascontiguousarray(kr)
    dl = np.ascontiguousarray(dl)
    dr = np.ascontiguousarray(dr)
    nm = L.oro_stereo_match(ext_l.h, ext_r.h, kl.ctypes.data, dl.ctypes.data, n, kr.ctypes.data, dr.ctypes.data,
                            len(kr), bf, fx, ur.ctypes.data, dp.ctypes.data)
    return ur[:n], dp[:n], nm


# ---- ORBmatcher oracle (oracle/orb_oracle_match.cpp): same snapshot structs as the product API ----
# int32_t (*)(void* ctx, int32_t idx1, int32_t idx2): the caller's epipolar test for a keypoint pair
EPIPOLAR_FN = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32)


def _match_sigs(L):
    vp, ci, cf = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    L.oro_sbp_local.argtypes = [vp, vp, vp, vp, ci, cf, ci, cf, cf]
    L.oro_sbp_lastframe.argtypes = [vp, vp, vp, vp, ci, cf, ci, ci, ci]
    L.oro_sbp_lastframe_stereo.argtypes = [vp, vp, vp, vp, vp, ci, cf, ci, ci, ci]
    L.oro_sbp_lastframe_pose.argtypes = [vp, vp, vp, vp, ci, vp, vp, vp, cf, ci, ci, ci]
    L.oro_sbp_kf.argtypes = [vp, vp, vp, ci, cf, ci, ci]
    L.oro_search_for_init.argtypes = [vp, vp, vp, vp, ci, cf, ci]
    L.oro_search_by_bow.argtypes = [vp, vp, vp, ci, vp, vp, vp, vp, cf, ci]
    L.oro_stereo_knn_ratio.argtypes = [vp, ci, vp, ci, cf, vp, vp]
    L.oro_search_by_bow_kf.argtypes = [vp, vp, vp, ci, vp, vp, vp, vp, ci, vp, vp, cf, ci]
    L.oro_distinctive_descriptors.argtypes = [vp, vp, ci, vp]
    L.oro_search_for_triangulation.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, ci, ci, ci, vp]
    L.oro_fuse.argtypes = [vp, vp, vp, vp, ci, cf, ci, vp, vp]
    L.oro_fuse_rig.argtypes = [vp, vp, vp, vp, vp, ci, cf, ci, ci, vp, vp]
    L.oro_search_by_bow_kf2.argtypes = [vp, vp, vp, ci, ci, vp, vp, vp, vp, ci, ci, vp, vp, cf, ci]
    L.oro_sbp_sim3.argtypes = [vp, vp, vp, ci, vp, ci, cf, vp, vp]
    L.oro_sbp_sim3_rig.argtypes = [vp, vp, vp, vp, ci, vp, ci, cf, vp, vp]
    L.oro_search_for_triangulation_epi.argtypes = [vp, vp, vp, vp, vp, vp, vp, ci, ci, EPIPOLAR_FN, vp, vp]
    L.oro_search_by_sim3.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, cf, vp, vp]
    L.oro_is_in_frustum.argtypes = [vp, vp, vp, ci, vp]
    L.oro_search_local_points.argtypes = [vp, vp, vp, ci, vp, vp, cf, ci, cf, cf, vp]
    L.oro_is_in_frustum_rig.argtypes = [vp, vp, vp, vp, ci, vp]
    L.oro_search_local_points_rig.argtypes = [vp, vp, vp, vp, ci, vp, vp, cf, ci, cf, cf, vp]
    return L


class OracleMatcher:
    """CPU restatement of ORBmatcher's Tracking-thread methods. Inputs are the product's snapshot
    objects (orb_slam3_ros_amd.matcher.MatchFrame / FeatureVector / record arrays); mvp arrays are
    updated in place exactly like the product API."""

    def __init__(self, nnratio=0.6, checkOri=True):
        self.L = _match_sigs(lib())
        self.nnratio, self.checkOri = float(nnratio), int(bool(checkOri))

    def sbp_local(self, F, mvp, mvp_obs, mps, th=3.0, bFar=False, thFar=50.0):
        return self.L.oro_sbp_local(F.ref(), mvp.ctypes.data, mvp_obs.ctypes.data, mps.ctypes.data, len(mps),
                                    float(th), int(bFar), float(thFar), self.nnratio)

    def sbp_lastframe(self, F, mvp, mvp_obs, pts, th, bForward, bBackward):
        return self.L.oro_sbp_lastframe(F.ref(), mvp.ctypes.data, mvp_obs.ctypes.data, pts.ctypes.data, len(pts),
                                        float(th), int(bForward), int(bBackward), self.checkOri)

    def sbp_lastframe_pose(self, F, mvp, mvp_obs, pts, Tcw, cam, th, bForward, bBackward, Trl=None):
        """pts: LAST_POINT records; Tcw / Trl: orbfe_pose structures; cam: orbfe_camera_model."""
        import ctypes
        return self.L.oro_sbp_lastframe_pose(F.ref(), mvp.ctypes.data, mvp_obs.ctypes.data, pts.ctypes.data, len(pts),
                                             ctypes.addressof(Tcw), ctypes.addressof(Trl) if Trl is not None else None,
                                             ctypes.addressof(cam), float(th), int(bForward), int(bBackward),
                                             self.checkOri)

    def sbp_lastframe_stereo(self, F, mvp, mvp_obs, pts, right_uv, th, bForward, bBackward):
        ruv = np.ascontiguousarray(right_uv, np.float32)
        return self.L.oro_sbp_lastframe_stereo(F.ref(), mvp.ctypes.data, mvp_obs.ctypes.data, pts.ctypes.data,
                                               ruv.ctypes.data, len(pts), float(th), int(bForward), int(bBackward),
                                               self.checkOri)

    def sbp_kf(self, F, mvp, pts, th, ORBdist):
        return self.L.oro_sbp_kf(F.ref(), mvp.ctypes.data, pts.ctypes.data, len(pts), float(th), int(ORBdist),
                                 self.checkOri)

    def search_for_init(self, F1, F2, prev, m12, windowSize=10):
        return self.L.oro_search_for_init(F1.ref(), F2.ref(), prev.ctypes.data, m12.ctypes.data, int(windowSize),
                                          self.nnratio, self.checkOri)

    def search_by_bow(self, kf_keys, kf_desc, kf_mp, kf_fv, F, f_fv):
        out = np.full(F.N, -1, np.int32)
        kk = np.ascontiguousarray(kf_keys)
        kd = np.ascontiguousarray(kf_desc, np.uint8)
        km = np.ascontiguousarray(kf_mp, np.int32)
        n = self.L.oro_search_by_bow(kk.ctypes.data, kd.ctypes.data, km.ctypes.data, len(km), kf_fv.ref(), F.ref(),
                                     f_fv.ref(), out.ctypes.data, self.nnratio, self.checkOri)
        return n, out

    def search_by_bow_kf(self, keys1, desc1, mp1, fv1, keys2, desc2, mp2, fv2, nleft1=-1, nleft2=-1):
        k1, k2 = np.ascontiguousarray(keys1), np.ascontiguousarray(keys2)
        d1 = np.ascontiguousarray(desc1, np.uint8)
        d2 = np.ascontiguousarray(desc2, np.uint8)
        m1 = np.ascontiguousarray(mp1, np.int32)
        m2 = np.ascontiguousarray(mp2, np.int32)
        out = np.full(len(k1), -1, np.int32)
        n = self.L.oro_search_by_bow_kf2(k1.ctypes.data, d1.ctypes.data, m1.ctypes.data, len(k1), int(nleft1),
                                         fv1.ref(), k2.ctypes.data, d2.ctypes.data, m2.ctypes.data, len(k2),
                                         int(nleft2), fv2.ref(), out.ctypes.data, self.nnratio, self.checkOri)
        return n, out


    def search_for_triangulation(self, KF1, mp1, fv1, KF2, mp2, fv2, F12, ep, level_sigma2_2, bOnlyStereo=False,
                                 bCoarse=False):
        m1 = np.ascontiguousarray(mp1, np.int32)
        m2 = np.ascontiguousarray(mp2, np.int32)
        F = np.ascontiguousarray(F12, np.float32).reshape(9)
        e = np.ascontiguousarray(ep, np.float32).reshape(2)
        sg = np.ascontiguousarray(level_sigma2_2, np.float32)
        out = np.full(KF1.N, -1, np.int32)
        n = self.L.oro_search_for_triangulation(KF1.ref(), m1.ctypes.data, fv1.ref(), KF2.ref(), m2.ctypes.data,
                                                fv2.ref(), F.ctypes.data, e.ctypes.data, sg.ctypes.data,
                                                int(bOnlyStereo), int(bCoarse), self.checkOri, out.ctypes.data)
        return n, out

    def fuse(self, KF, cam, pts, th=3.0, inv_level_sigma2=None, sim3=False, model=None, bRight=False):
        if inv_level_sigma2 is None:
            sf = KF.scale_factors
            inv_level_sigma2 = (np.float32(1.0) / (sf * sf)).astype(np.float32)
        sig = np.ascontiguousarray(inv_level_sigma2, np.float32)
        p = np.ascontiguousarray(pts)
        bi = np.full(len(p), -1, np.int32)
        bd = np.full(len(p), -1, np.int32)
        n = self.L.oro_fuse_rig(KF.ref(), ctypes.byref(cam), ctypes.byref(model) if model is not None else None,
                                sig.ctypes.data, p.ctypes.data, len(p), float(th), int(bool(sim3)), int(bool(bRight)),
                                bi.ctypes.data, bd.ctypes.data)
        return n, bi, bd

    def sbp_sim3(self, KF, cam, pts, matched, th=10, ratioHamming=1.0, point_kfs=None, matched_kf=None, model=None):
        p = np.ascontiguousarray(pts)
        pk = None if point_kfs is None else np.ascontiguousarray(point_kfs, np.int32)
        return self.L.oro_sbp_sim3_rig(KF.ref(), ctypes.byref(cam), None if model is None else ctypes.byref(model),
                                       p.ctypes.data, len(p), None if pk is None else pk.ctypes.data, int(th),
                                       float(ratioHamming), matched.ctypes.data,
                                       None if matched_kf is None else matched_kf.ctypes.data)

    def search_for_triangulation_epi(self, KF1, mp1, fv1, KF2, mp2, fv2, ep, epi, bOnlyStereo=False):
        """SearchForTriangulation with bCoarse false, the epipolar test delegated to epi(idx1, idx2) -> bool
        (pCamera1->epipolarConstrain for that keypoint pair)."""
        m1 = np.ascontiguousarray(mp1, np.int32)
        m2 = np.ascontiguousarray(mp2, np.int32)
        e = np.ascontiguousarray(ep, np.float32).reshape(2)
        out = np.full(KF1.N, -1, np.int32)
        cb = EPIPOLAR_FN(lambda ctx, i1, i2: 1 if epi(i1, i2) else 0)
        n = self.L.oro_search_for_triangulation_epi(KF1.ref(), m1.ctypes.data, fv1.ref(), KF2.ref(), m2.ctypes.data,
                                                    fv2.ref(), e.ctypes.data, int(bOnlyStereo), self.checkOri, cb,
                                                    None, out.ctypes.data)
        return n, out

    def search_by_sim3(self, KF1, KF2, pts1, pts2, cam1, cam2, S12, S21, th, matches12, matched_idx2=None):
        p1, p2 = np.ascontiguousarray(pts1), np.ascontiguousarray(pts2)
        mi = None if matched_idx2 is None else np.ascontiguousarray(matched_idx2, np.int32)
        return self.L.oro_search_by_sim3(KF1.ref(), KF2.ref(), p1.ctypes.data, p2.ctypes.data, ctypes.byref(cam1),
                                         ctypes.byref(cam2), ctypes.byref(S12), ctypes.byref(S21), float(th),
                                         matches12.ctypes.data, None if mi is None else mi.ctypes.data)


def distinctive_descriptors(desc, offsets):
    L = _match_sigs(lib())
    d = np.ascontiguousarray(desc, np.uint8)
    o = np.ascontiguousarray(offsets, np.int32)
    best = np.full(len(o) - 1, -1, np.int32)
    L.oro_distinctive_descriptors(d.ctypes.data, o.ctypes.data, len(o) - 1, best.ctypes.data)
    return best


def is_in_frustum(F, cam, pts3d, rig=None):
    """(nToMatch, tracking records) — the caller passes MAP_POINT_DTYPE / MAP_POINT_3D_DTYPE arrays;
    rig: a StereoRig (camera models, right view) or None (pinhole from cam)."""
    from orb_slam3_ros_amd.matcher import MAP_POINT_DTYPE
    L = _match_sigs(lib())
    pts = np.ascontiguousarray(pts3d)
    track = np.zeros(len(pts), MAP_POINT_DTYPE)
    n = L.oro_is_in_frustum_rig(F.ref(), ctypes.byref(cam), ctypes.byref(rig) if rig is not None else None,
                                pts.ctypes.data, len(pts), track.ctypes.data)
    return n, track


def search_local_points(F, cam, pts3d, mvp, mvp_obs, th=1.0, bFar=False, thFar=50.0, nnratio=0.8, rig=None):
    L = _match_sigs(lib())
    pts = np.ascontiguousarray(pts3d)
    ntm = ctypes.c_int32(0)
    n = L.oro_search_local_points_rig(F.ref(), ctypes.byref(cam), ctypes.byref(rig) if rig is not None else None,
                                      pts.ctypes.data, len(pts), mvp.ctypes.data, mvp_obs.ctypes.data, float(th),
                                      int(bFar), float(thFar), float(nnratio), ctypes.byref(ntm))
    return n, int(ntm.value)


def stereo_knn_ratio(left_desc, right_desc, ratio=0.7):
    L = _match_sigs(lib())
    a = np.ascontiguousarray(left_desc, np.uint8).reshape(-1, 32)
    b = np.ascontiguousarray(right_desc, np.uint8).reshape(-1, 32)
    t = np.full(len(a), -1, np.int32)
    d = np.full(len(a), -1, np.int32)
    g = L.oro_stereo_knn_ratio(a.ctypes.data, len(a), b.ctypes.data, len(b), float(ratio), t.ctypes.data,
                               d.ctypes.data)
    return g, t, d


# ---- DBoW2 vocabulary oracle (oracle/orb_oracle_bow.cpp) ----
class OracleVocabulary:
    def __init__(self, handle):
        self.L_ = lib()
        self.h = handle

    @staticmethod
    def _lib():
        L = lib()
        vp, ci = ctypes.c_void_p, ctypes.c_int
        L.oro_voc_create.restype = vp
        L.oro_voc_create.argtypes = [ci, ci, ci, ci, ci, vp, vp, vp, vp]
        L.oro_voc_load_bin.restype = vp
        L.oro_voc_load_bin.argtypes = [vp, ctypes.c_size_t]
        L.oro_voc_destroy.argtypes = [vp]
        L.oro_voc_transform.argtypes = [vp, vp, ci, ci, vp, vp, vp, vp, vp, vp, vp]
        return L

    @classmethod
    def from_arrays(cls, k, Lv, scoring, weighting, parents, is_leaf, desc, weights):
        L = cls._lib()
        par = np.ascontiguousarray(parents, np.int32)
        leaf = np.ascontiguousarray(is_leaf, np.uint8)
        d = np.ascontiguousarray(desc, np.uint8)
        w = np.ascontiguousarray(weights, np.float64)
        o = cls(L.oro_voc_create(k, Lv, scoring, weighting, len(par), par.ctypes.data, leaf.ctypes.data,
                                 d.ctypes.data, w.ctypes.data))
        o._keep = (par, leaf, d, w)
        return o

    @classmethod
    def from_bin(cls, data):
        L = cls._lib()
        buf = np.frombuffer(data, np.uint8)
        h = L.oro_voc_load_bin(buf.ctypes.data, len(buf))
        return cls(h) if h else None

    def transform(self, desc, levelsup=4):
        L = self._lib()
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(d)
        bid = np.zeros(max(n, 1), np.uint32)
        bw = np.zeros(max(n, 1), np.float64)
        fid = np.zeros(max(n, 1), np.uint32)
        foff = np.zeros(n + 1, np.int32)
        fidx = np.zeros(max(n, 1), np.uint32)
        nb, nf = ctypes.c_int(), ctypes.c_int()
        L.oro_voc_transform(self.h, d.ctypes.data, n, levelsup, bid.ctypes.data, bw.ctypes.data, ctypes.byref(nb),
                            fid.ctypes.data, foff.ctypes.data, fidx.ctypes.data, ctypes.byref(nf))
        return (bid[:nb.value].copy(), bw[:nb.value].copy()), (fid[:nf.value].copy(), foff[:nf.value + 1].copy(),
                                                               fidx[:foff[nf.value]].copy())

    def __del__(self):
        try:
            if self.h:
                self._lib().oro_voc_destroy(self.h)
        except Exception:
            pass


def remap_linear(src, mapx, mapy):
    L = lib()
    L.oro_remap_linear.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    src = np.ascontiguousarray(src, np.uint8)
    mapx = np.ascontiguousarray(mapx, np.float32)
    mapy = np.ascontiguousarray(mapy, np.float32)
    dh, dw = mapx.shape
    out = np.zeros((dh, dw), np.uint8)
    L.oro_remap_linear(src.ctypes.data, src.shape[1], src.shape[0], src.strides[0], mapx.ctypes.data,
                       mapy.ctypes.data, dw, dh, out.ctypes.data, dw)
    return out


def remap_bilinear_tab():
    L = lib()
    L.oro_remap_bilinear_tab.argtypes = [ctypes.c_void_p]
    t = np.zeros((32 * 32, 4), np.int16)
    L.oro_remap_bilinear_tab(t.ctypes.data)
    return t


def undistort_points(pts, K4, dist):
    L = lib()
    L.oro_undistort_points.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                       ctypes.c_void_p]
    p = np.ascontiguousarray(pts, np.float32).reshape(-1, 2)
    k = np.ascontiguousarray(K4, np.float32).reshape(4)
    d = np.ascontiguousarray(dist, np.float32).reshape(-1)
    out = np.zeros_like(p)
    L.oro_undistort_points(p.ctypes.data, len(p), k.ctypes.data, d.ctypes.data, len(d), out.ctypes.data)
    return out
