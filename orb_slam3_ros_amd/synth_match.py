"""Seeded synthetic matcher workloads (no datasets offline), SURVEY.md §8c "Config 5".

Frames get uniform keypoints with octaves in the extractor's per-level budget proportions, random
angles and descriptors; map points / projected points are a mix of noisy COPIES of frame
features (descriptor bits flipped with probability p, i.e. Binomial(256, p) flips, projected near
the source keypoint so the ratio tests, "already matched" skips and rotation histogram all fire)
and uniformly placed random ones. Used by the parity tests and bench.py's matcher line.
"""
from __future__ import annotations

import numpy as np

from .extractor import KEYPOINT_DTYPE
from .matcher import (MAP_POINT_3D_DTYPE, MAP_POINT_DTYPE, MP_BAD, MP_IN_VIEW, MP_IN_VIEW_R, MP_SKIP, PROJ_POINT_DTYPE, Camera,
                      FeatureVector, KFCamera, MatchFrame, Pose)


def scale_factors(nlevels: int = 8, scale_factor: float = 1.2) -> np.ndarray:
    """mvScaleFactor (ORBextractor.cc:414-420): running float product."""
    s = np.ones(nlevels, np.float32)
    for i in range(1, nlevels):
        s[i] = np.float32(s[i - 1] * np.float32(scale_factor))
    return s


def level_weights(nlevels: int = 8, scale_factor: float = 1.2) -> np.ndarray:
    w = (1.0 / scale_factor) ** np.arange(nlevels)
    return w / w.sum()


def flip_bits(rng, desc: np.ndarray, p: float) -> np.ndarray:
    bits = np.unpackbits(desc.reshape(-1, 32), axis=1)
    bits ^= (rng.random(bits.shape) < p).astype(np.uint8)
    return np.packbits(bits, axis=1)


def synth_frame(rng, n: int, w: int = 752, h: int = 480, nlevels: int = 8, stereo: bool = True,
                mbf: float = 0.110078 * 458.654) -> MatchFrame:
    k = np.zeros(n, KEYPOINT_DTYPE)
    k["x"] = rng.uniform(0, w - 1, n).astype(np.float32)
    k["y"] = rng.uniform(0, h - 1, n).astype(np.float32)
    k["octave"] = rng.choice(nlevels, n, p=level_weights(nlevels))
    sf = scale_factors(nlevels)
    k["size"] = (31.0 * sf[k["octave"]]).astype(np.float32)
    k["angle"] = rng.uniform(0, 360, n).astype(np.float32)
    k["response"] = rng.integers(7, 100, n).astype(np.float32)
    k["class_id"] = -1
    desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    ur = None
    if stereo:
        ur = np.where(rng.random(n) < 0.7, k["x"] - rng.uniform(0, 60, n), -1.0).astype(np.float32)
    return MatchFrame(k, desc, (0.0, float(w), 0.0, float(h)), sf, ur, mbf)


def perturbed_frame(rng, F: MatchFrame, shift=(4.0, -3.0), jitter: float = 1.0, rot: float = 10.0,
                    flip_p: float = 0.05, drop: float = 0.1):
    """Another view of F: keypoints shifted/jittered, angles rotated, descriptors noisy, some
    replaced by new random features (the second frame of SearchForInitialization etc.).
    Returns (frame, src): src[i] = index of the F feature that keypoint i copies, -1 if new."""
    n = F.N
    k = F.keys.copy()
    k["x"] = np.clip(k["x"] + shift[0] + rng.normal(0, jitter, n), 0, F.bounds[1] - 1).astype(np.float32)
    k["y"] = np.clip(k["y"] + shift[1] + rng.normal(0, jitter, n), 0, F.bounds[3] - 1).astype(np.float32)
    k["angle"] = np.mod(k["angle"] + rot + rng.normal(0, 3.0, n), 360.0).astype(np.float32)
    desc = flip_bits(rng, F.desc, flip_p)
    new = rng.random(n) < drop
    desc[new] = rng.integers(0, 256, (int(new.sum()), 32), dtype=np.uint8)
    perm = rng.permutation(n)   # the other frame's keypoint order is unrelated
    ur = None if F.uright is None else F.uright[perm] + np.float32(shift[0])
    src = np.where(new, -1, np.arange(n))[perm]
    return MatchFrame(k[perm], desc[perm], F.bounds, F.scale_factors, ur, F.mbf), src


def synth_local_map(rng, F: MatchFrame, n_mps: int, copy_frac: float = 0.3, flip_p: float = 0.05,
                    copy_near: bool = True, nlevels: int = 8) -> np.ndarray:
    """Config 5 map points: mbTrackInView mostly set, projX/Y uniform (copies: near their source),
    projXR = projX - U(0,60) (copies with a stereo source: that source's uR +- 1), level by budget,
    viewCos in U(0.99, 1)."""
    m = np.zeros(n_mps, MAP_POINT_DTYPE)
    w, h = F.bounds[1], F.bounds[3]
    m["proj_x"] = rng.uniform(0, w, n_mps)
    m["proj_y"] = rng.uniform(0, h, n_mps)
    m["proj_xr"] = m["proj_x"] - rng.uniform(0, 60, n_mps)
    m["view_cos"] = rng.uniform(0.99, 1.0, n_mps)
    m["depth"] = rng.uniform(0.5, 60.0, n_mps)
    m["scale_level"] = rng.choice(nlevels, n_mps, p=level_weights(nlevels))
    fl = np.full(n_mps, MP_IN_VIEW, np.int32)
    fl[rng.random(n_mps) < 0.05] = 0
    fl[rng.random(n_mps) < 0.02] |= MP_BAD
    m["flags"] = fl
    m["observations"] = np.where(rng.random(n_mps) < 0.1, 0, rng.integers(1, 20, n_mps))
    m["id"] = np.arange(n_mps) + 1000
    m["desc"] = rng.integers(0, 256, (n_mps, 32), dtype=np.uint8)
    if F.N:
        cp = np.nonzero(rng.random(n_mps) < copy_frac)[0]
        src = rng.integers(0, F.N, len(cp))
        m["desc"][cp] = flip_bits(rng, F.desc[src], flip_p)
        if copy_near:
            m["proj_x"][cp] = F.keys["x"][src] + rng.normal(0, 1.5, len(cp))
            m["proj_y"][cp] = F.keys["y"][src] + rng.normal(0, 1.5, len(cp))
            m["scale_level"][cp] = F.keys["octave"][src]
            if F.uright is not None:
                ur = F.uright[src]
                m["proj_xr"][cp] = np.where(ur > 0, ur + rng.uniform(-1, 1, len(cp)), m["proj_xr"][cp])
    return m


def initial_slots(rng, n: int, frac: float = 0.1):
    """Pre-existing F.mvpMapPoints handles and their Observations() (some zero)."""
    mvp = np.full(n, -1, np.int32)
    obs = np.zeros(n, np.int32)
    sel = rng.random(n) < frac
    mvp[sel] = rng.integers(1, 900, int(sel.sum()))
    obs[sel] = np.where(rng.random(int(sel.sum())) < 0.4, 0, rng.integers(1, 10, int(sel.sum())))
    return mvp, obs


def synth_proj_points(rng, F: MatchFrame, n: int, copy_frac: float = 0.8, flip_p: float = 0.05, rot: float = 15.0,
                      invalid: float = 0.1, behind: float = 0.02) -> np.ndarray:
    """Projected last-frame / keyframe points: copies land near a current keypoint with its
    octave (+-1) and angle + rot (+ noise, some outliers); the rest are random."""
    p = np.zeros(n, PROJ_POINT_DTYPE)
    w, h = F.bounds[1], F.bounds[3]
    p["u"] = rng.uniform(-20, w + 20, n)
    p["v"] = rng.uniform(-20, h + 20, n)
    p["invzc"] = np.where(rng.random(n) < behind, -0.1, 1.0 / rng.uniform(1, 30, n))
    p["octave"] = rng.integers(0, len(F.scale_factors), n)
    p["angle"] = rng.uniform(0, 360, n)
    p["valid"] = (rng.random(n) >= invalid).astype(np.int32)
    p["observations"] = np.where(rng.random(n) < 0.1, 0, rng.integers(1, 20, n))
    p["id"] = np.arange(n) + 5000
    p["desc"] = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    if F.N:
        cp = np.nonzero(rng.random(n) < copy_frac)[0]
        src = rng.integers(0, F.N, len(cp))
        p["desc"][cp] = flip_bits(rng, F.desc[src], flip_p)
        p["u"][cp] = F.keys["x"][src] + rng.normal(0, 2.0, len(cp))
        p["v"][cp] = F.keys["y"][src] + rng.normal(0, 2.0, len(cp))
        p["octave"][cp] = np.clip(F.keys["octave"][src] + rng.integers(-1, 2, len(cp)), 0,
                                  len(F.scale_factors) - 1)
        outl = rng.random(len(cp)) < 0.15
        p["angle"][cp] = np.mod(np.where(outl, rng.uniform(0, 360, len(cp)),
                                         F.keys["angle"][src] + rot + rng.normal(0, 4, len(cp))), 360.0)
        if F.uright is not None:   # keep invzc consistent with the stereo check for stereo sources
            ur = F.uright[src]
            iz = (p["u"][cp] - ur) / np.float32(F.mbf)
            p["invzc"][cp] = np.where((ur > 0) & (iz > 0), iz, p["invzc"][cp])
    return p


def synth_bow(rng, n_words: int, kf: MatchFrame, F: MatchFrame, shared_src=None):
    """Node assignment for both frames (a feature's node = the vocabulary node at the FeatureVector
    level). Features of F that are noisy copies of KF features (shared_src[i] = KF index or -1)
    share their source's node."""
    wk = rng.integers(0, n_words, kf.N)
    wf = rng.integers(0, n_words, F.N)
    if shared_src is not None:
        m = shared_src >= 0
        wf[m] = wk[shared_src[m]]

    def fv(words):
        d = {}
        for i, wd in enumerate(words.tolist()):
            d.setdefault(int(wd) * 7 + 3, []).append(i)   # sparse node ids
        return FeatureVector(d)

    return fv(wk), fv(wf)


def synth_kf_pair(rng, n1, words, rot=20.0, drop=0.15):
    """Two keyframes sharing a scene: KF2 = perturbed copy of KF1 (dropped / extra points,
    rotated angles), map-point handles with NULL / bad (-1) slots on both sides."""
    K1 = synth_frame(rng, n1, stereo=False)
    K2, src = perturbed_frame(rng, K1, rot=rot, flip_p=0.05, drop=drop)
    mp1 = np.where(rng.random(K1.N) < 0.2, -1, np.arange(K1.N) + 10).astype(np.int32)
    mp2 = np.where(rng.random(K2.N) < 0.2, -1, np.arange(K2.N) + 5000).astype(np.int32)
    fv1, fv2 = synth_bow(rng, words, K1, K2, src)
    return K1, K2, mp1, mp2, fv1, fv2


def synth_distinctive_sets(rng, sizes, flip_p=0.2):
    """Per-map-point observation descriptor sets (noisy copies of one descriptor) with duplicate
    rows (equal medians: the first row must win)."""
    sets = []
    for N in sizes:
        if N == 0:
            sets.append(np.zeros((0, 32), np.uint8))
            continue
        base = rng.integers(0, 256, 32, dtype=np.uint8)
        d = flip_bits(rng, np.repeat(base[None], N, 0), flip_p)
        if N >= 4:
            d[1] = d[3]
        sets.append(d)
    return sets


def synth_camera(rng, fx=458.654, fy=457.296, cx=367.215, cy=248.375, rot_deg=10.0):
    """A random pose (rotation of up to rot_deg about a random axis, translation ~1 m)."""
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    ang = np.deg2rad(rng.uniform(-rot_deg, rot_deg))
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    R = np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K
    t = rng.normal(scale=1.0, size=3)
    return Camera.make(R, t, fx, fy, cx, cy)


def synth_local_map_3d(rng, F: MatchFrame, cam: Camera, n: int, copy_frac: float = 0.5, flip_p: float = 0.05,
                       nlevels: int = 8, scale_factor: float = 1.2) -> np.ndarray:
    """Local map points in the world: they project near frame keypoints (copies, predicted level =
    the keypoint's octave) or anywhere around the image; a few are behind the camera, outside the
    scale-invariance distance range, seen at a grazing angle, bad, or already seen this frame."""
    R = np.array(cam.Rcw[:], np.float64).reshape(3, 3)
    t = np.array(cam.tcw[:], np.float64)
    w, h = F.bounds[1], F.bounds[3]
    u = rng.uniform(-60, w + 60, n)
    v = rng.uniform(-60, h + 60, n)
    lvl = rng.choice(nlevels, n, p=level_weights(nlevels))
    desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    if F.N:
        cp = np.nonzero(rng.random(n) < copy_frac)[0]
        src = rng.integers(0, F.N, len(cp))
        u[cp] = F.keys["x"][src] + rng.normal(0, 1.0, len(cp))
        v[cp] = F.keys["y"][src] + rng.normal(0, 1.0, len(cp))
        lvl[cp] = F.keys["octave"][src]
        desc[cp] = flip_bits(rng, F.desc[src], flip_p)
    z = rng.uniform(0.5, 40.0, n)
    z[rng.random(n) < 0.02] *= -1.0
    Pc = np.stack([(u - cam.cx) * z / cam.fx, (v - cam.cy) * z / cam.fy, z], 1)
    P = (Pc - t) @ R                       # R^T (Pc - t), row-vector form
    dist = np.linalg.norm(Pc, axis=1)
    # PredictScale(dist) = ceil(log(max/dist) / log(sf)) = lvl  <=>  max = dist * sf^(lvl - frac)
    max_d = dist * scale_factor ** (lvl - rng.uniform(0.1, 0.9, n))
    out = rng.random(n) < 0.08
    max_d[out] *= rng.choice([0.5, 2.5], int(out.sum()))
    min_d = max_d / scale_factor ** (nlevels - 1)
    view = P - np.array(cam.Ow[:], np.float64)
    view /= np.maximum(np.linalg.norm(view, axis=1, keepdims=True), 1e-9)
    nrm = view + rng.normal(0, 0.3, (n, 3))
    graze = rng.random(n) < 0.05
    nrm[graze] = -nrm[graze]
    nrm /= np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-9)
    m = np.zeros(n, MAP_POINT_3D_DTYPE)
    m["pos"] = P.astype(np.float32)
    m["normal"] = nrm.astype(np.float32)
    m["min_dist"] = min_d.astype(np.float32)
    m["max_dist"] = max_d.astype(np.float32)
    fl = np.zeros(n, np.int32)
    fl[rng.random(n) < 0.03] |= MP_BAD
    fl[rng.random(n) < 0.03] |= MP_SKIP
    m["flags"] = fl
    m["observations"] = np.where(rng.random(n) < 0.1, 0, rng.integers(1, 20, n))
    m["id"] = np.arange(n) + 20000
    m["desc"] = desc
    return m


# ---- back-end scenes ----
def _rand_rotation(rng, rot_deg):
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    ang = np.deg2rad(rng.uniform(-rot_deg, rot_deg))
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K


def synth_kf_camera(rng, fx=458.654, fy=457.296, cx=367.215, cy=248.375, rot_deg=10.0) -> KFCamera:
    R = _rand_rotation(rng, rot_deg)
    t = rng.normal(scale=1.0, size=3)
    return KFCamera.make(Pose.se3(R, t), fx, fy, cx, cy)


def synth_fuse_scene(rng, n_kp: int, n_pts: int, dup: int = 1, copy_frac: float = 0.6):
    """A keyframe, its camera and map points that project near its keypoints (for Fuse and
    SearchByProjection(Sim3)). dup > 1 makes several points compete for the same keypoints.
    The stereo keypoints that points were copied from get a consistent mvuRight."""
    KF = synth_frame(rng, n_kp, stereo=True)
    cam = synth_kf_camera(rng)
    R = cam.Tcw.rotation()
    c = Camera.make(R, np.array(cam.Tcw.t[:], np.float64), cam.fx, cam.fy, cam.cx, cam.cy)
    base = synth_local_map_3d(rng, KF, c, max(n_pts // dup, 1), copy_frac=copy_frac)
    pts = np.concatenate([base] * dup)[:n_pts].copy()
    if dup > 1:   # jitter the duplicates so they are distinct points with the same neighbourhood
        pts["pos"] += rng.normal(0, 1e-3, pts["pos"].shape).astype(np.float32)
        pts["desc"] = flip_bits(rng, pts["desc"], 0.03)
    pts["id"] = np.arange(len(pts)) + 20000
    # consistent right coordinates for the keypoints nearest to a projected point
    P = pts["pos"].astype(np.float64)
    t = np.array(cam.Tcw.t[:], np.float64)
    Pc = P @ R.T + t
    ok = Pc[:, 2] > 0.1
    u = cam.fx * Pc[ok, 0] / Pc[ok, 2] + cam.cx
    v = cam.fy * Pc[ok, 1] / Pc[ok, 2] + cam.cy
    ur_pt = u - KF.mbf / Pc[ok, 2]
    if KF.uright is not None and ok.any():
        d2 = (KF.keys["x"][:, None] - u[None, :]) ** 2 + (KF.keys["y"][:, None] - v[None, :]) ** 2
        j = d2.argmin(1)
        near = (d2[np.arange(KF.N), j] < 4.0) & (KF.uright >= 0)
        KF.uright[near] = (ur_pt[j[near]] + rng.normal(0, 0.5, int(near.sum()))).astype(np.float32)
    return KF, cam, pts


def synth_sim3_pair(rng, n1: int, extra2: float = 0.2, scale: float = 1.0, nlevels: int = 8, sf: float = 1.2):
    """Two keyframes looking at the same points (SearchBySim3 / SearchForTriangulation). Returns
    (KF1, KF2, pts1, pts2, cam1, cam2, S12, S21, src) with src[j] = the KF1 keypoint KF2 keypoint j
    observes (-1 if new). S12 maps camera-2 coordinates to camera 1 (scaled by `scale`)."""
    fx, fy, cx, cy, w, h = 458.654, 457.296, 367.215, 248.375, 752, 480
    R1 = _rand_rotation(rng, 5.0)
    t1 = rng.normal(scale=0.5, size=3)
    dR = _rand_rotation(rng, 8.0)
    R2 = dR @ R1
    t2 = t1 + rng.normal(scale=0.3, size=3)
    cam1 = KFCamera.make(Pose.se3(R1, t1), fx, fy, cx, cy)
    cam2 = KFCamera.make(Pose.se3(R2, t2), fx, fy, cx, cy)
    KF1 = synth_frame(rng, n1, stereo=False)
    u1, v1 = KF1.keys["x"].astype(np.float64), KF1.keys["y"].astype(np.float64)
    z1 = rng.uniform(1.0, 12.0, n1)
    Pc1 = np.stack([(u1 - cx) * z1 / fx, (v1 - cy) * z1 / fy, z1], 1)
    Pw = (Pc1 - t1) @ R1
    Pc2 = Pw @ R2.T + t2
    o1 = KF1.keys["octave"].astype(np.float64)
    max_d = z1 * np.sqrt(1 + ((u1 - cx) / fx) ** 2 + ((v1 - cy) / fy) ** 2) * sf ** (o1 - 0.5)
    d2 = np.linalg.norm(Pc2, axis=1)
    pred2 = np.clip(np.ceil(np.log(max_d / d2) / np.log(sf)), 0, nlevels - 1).astype(np.int32)
    u2 = fx * Pc2[:, 0] / Pc2[:, 2] + cx + rng.normal(0, 0.7, n1)
    v2 = fy * Pc2[:, 1] / Pc2[:, 2] + cy + rng.normal(0, 0.7, n1)
    vis = (Pc2[:, 2] > 0) & (u2 >= 0) & (u2 < w) & (v2 >= 0) & (v2 < h) & (rng.random(n1) < 0.85)
    idx = np.nonzero(vis)[0]
    n_new = int(len(idx) * extra2)
    n2 = len(idx) + n_new
    k2 = np.zeros(n2, KEYPOINT_DTYPE)
    k2["x"][:len(idx)] = u2[idx]
    k2["y"][:len(idx)] = v2[idx]
    k2["octave"][:len(idx)] = np.maximum(pred2[idx] - (rng.random(len(idx)) < 0.3), 0)
    k2["x"][len(idx):] = rng.uniform(0, w - 1, n_new)
    k2["y"][len(idx):] = rng.uniform(0, h - 1, n_new)
    k2["octave"][len(idx):] = rng.choice(nlevels, n_new, p=level_weights(nlevels))
    sfs = scale_factors(nlevels)
    k2["size"] = (31.0 * sfs[k2["octave"]]).astype(np.float32)
    k2["angle"] = np.mod(np.concatenate([KF1.keys["angle"][idx], rng.uniform(0, 360, n_new)]) + 15.0, 360.0)
    k2["response"] = 20.0
    k2["class_id"] = -1
    d2desc = np.concatenate([flip_bits(rng, KF1.desc[idx], 0.06),
                             rng.integers(0, 256, (n_new, 32), dtype=np.uint8)])
    perm = rng.permutation(n2)
    src = np.concatenate([idx, np.full(n_new, -1)])[perm]
    KF2 = MatchFrame(k2[perm], d2desc[perm], (0.0, float(w), 0.0, float(h)), sfs, None, KF1.mbf)
    # map points: KF1's (some NULL / bad) and KF2's (the same point for observed ones)
    normal = Pw - np.array(cam1.Ow[:], np.float64)
    normal /= np.linalg.norm(normal, axis=1, keepdims=True)
    pts1 = np.zeros(n1, MAP_POINT_3D_DTYPE)
    pts1["pos"] = Pw.astype(np.float32)
    pts1["normal"] = normal.astype(np.float32)
    pts1["max_dist"] = max_d.astype(np.float32)
    pts1["min_dist"] = (max_d / sf ** (nlevels - 1)).astype(np.float32)
    pts1["desc"] = KF1.desc
    pts1["observations"] = 2
    pts1["id"] = np.where(rng.random(n1) < 0.15, -1, np.arange(n1) + 1000)
    pts1["flags"] = np.where(rng.random(n1) < 0.03, MP_BAD, 0)
    pts2 = np.zeros(n2, MAP_POINT_3D_DTYPE)
    has = src >= 0
    pts2[has] = pts1[src[has]]
    pts2["id"][has] = np.where(rng.random(int(has.sum())) < 0.1, -1, pts1["id"][src[has]] + 500000)
    pts2["id"][~has] = -1
    pts2["desc"] = KF2.desc
    R12 = R1 @ R2.T
    t12 = t1 - R12 @ t2
    S12 = Pose.sim3(R12, t12 * scale, scale)
    S21 = Pose.sim3(R12.T, -(R12.T @ (t12 * scale)) / scale, 1.0 / scale)
    return KF1, KF2, pts1, pts2, cam1, cam2, S12, S21, src


def fundamental_12(cam1: KFCamera, cam2: KFCamera):
    """F12 = K1^-T [t12]x R12 K2^-1 and the epipole ep = project2(T2w * Cw1) (ORBmatcher.cc:914-920,
    Pinhole.cpp:107-112), computed in float64 and rounded to float."""
    R1, R2 = cam1.Tcw.rotation(), cam2.Tcw.rotation()
    t1, t2 = np.array(cam1.Tcw.t[:], np.float64), np.array(cam2.Tcw.t[:], np.float64)
    R12 = R1 @ R2.T
    t12 = t1 - R12 @ t2
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]])
    K1 = np.array([[cam1.fx, 0, cam1.cx], [0, cam1.fy, cam1.cy], [0, 0, 1]])
    K2 = np.array([[cam2.fx, 0, cam2.cx], [0, cam2.fy, cam2.cy], [0, 0, 1]])
    F12 = np.linalg.inv(K1.T) @ tx @ R12 @ np.linalg.inv(K2)
    Cw = -(R1.T @ t1)
    C2 = R2 @ Cw + t2
    ep = np.array([cam2.fx * C2[0] / C2[2] + cam2.cx, cam2.fy * C2[1] / C2[2] + cam2.cy])
    return F12.astype(np.float32), ep.astype(np.float32)


# ---- two-camera (KannalaBrandt8 stereo, Frame.Nleft != -1) workloads, config 4's tracking path ----
def synth_frame_two(rng, nl: int, nr: int, w: int = 512, h: int = 512, nlevels: int = 8, stereo_frac: float = 0.5,
                    flip_p: float = 0.04) -> MatchFrame:
    """mvKeys (nl) ++ mvKeysRight (nr) on a w x h fisheye pair. A stereo_frac share of the left
    features has a right partner (a noisy copy a few pixels to the left, same octave):
    mvLeftToRightMatch / mvRightToLeftMatch link them both ways."""
    L = synth_frame(rng, nl, w, h, nlevels, stereo=False)
    R = synth_frame(rng, nr, w, h, nlevels, stereo=False)
    keys = np.concatenate([L.keys, R.keys])
    desc = np.concatenate([L.desc, R.desc])
    l2r = np.full(nl, -1, np.int32)
    r2l = np.full(nr, -1, np.int32)
    npair = int(min(nl, nr) * stereo_frac)
    if npair:
        li = rng.choice(nl, npair, replace=False)
        ri = rng.choice(nr, npair, replace=False)
        l2r[li] = ri
        r2l[ri] = li
        k = keys[nl + ri]
        k["x"] = np.clip(keys["x"][li] - rng.uniform(2, 40, npair), 0, w - 1).astype(np.float32)
        k["y"] = np.clip(keys["y"][li] + rng.normal(0, 1.0, npair), 0, h - 1).astype(np.float32)
        k["octave"] = keys["octave"][li]
        k["angle"] = np.mod(keys["angle"][li] + rng.normal(0, 2.0, npair), 360.0).astype(np.float32)
        keys[nl + ri] = k
        desc[nl + ri] = flip_bits(rng, desc[li], flip_p)
    return MatchFrame(keys, desc, L.bounds, L.scale_factors, None, L.mbf, nleft=nl, l2r=l2r, r2l=r2l)


def synth_local_map_two(rng, F: MatchFrame, n_mps: int, copy_frac: float = 0.5, flip_p: float = 0.05,
                        nlevels: int = 8) -> np.ndarray:
    """Map points seen by a two-camera frame: left view fields as synth_local_map, plus
    mbTrackInViewR / mTrackProjXR, YR / mTrackViewCosR / mnTrackScaleLevelR. Copies of a right
    feature project next to it in the right camera (and next to its left partner, if any)."""
    nl = F.nleft
    m = synth_local_map(rng, F, n_mps, copy_frac=0.0, flip_p=flip_p, nlevels=nlevels)
    w, h = F.bounds[1], F.bounds[3]
    m["proj_xr"] = rng.uniform(0, w, n_mps)
    m["proj_yr"] = rng.uniform(0, h, n_mps)
    m["view_cos_r"] = rng.uniform(0.99, 1.0, n_mps)
    m["scale_level_r"] = np.where(rng.random(n_mps) < 0.05, -1, rng.choice(nlevels, n_mps, p=level_weights(nlevels)))
    fl = m["flags"].copy()
    inr = rng.random(n_mps) < 0.8
    fl = np.where(inr, fl | MP_IN_VIEW_R, fl)
    fl = np.where(rng.random(n_mps) < 0.15, fl & ~MP_IN_VIEW, fl)   # seen by the right camera only
    m["flags"] = fl.astype(np.int32)
    if F.N:
        cp = np.nonzero(rng.random(n_mps) < copy_frac)[0]
        src = rng.integers(0, F.N, len(cp))
        m["desc"][cp] = flip_bits(rng, F.desc[src], flip_p)
        left = src < nl
        # left source: left view near it, right view near its partner (or random)
        li = cp[left]
        ls = src[left]
        m["proj_x"][li] = F.keys["x"][ls] + rng.normal(0, 1.5, len(li))
        m["proj_y"][li] = F.keys["y"][ls] + rng.normal(0, 1.5, len(li))
        m["scale_level"][li] = F.keys["octave"][ls]
        part = F.l2r[ls]
        hp = part >= 0
        m["proj_xr"][li[hp]] = F.keys["x"][nl + part[hp]] + rng.normal(0, 1.5, int(hp.sum()))
        m["proj_yr"][li[hp]] = F.keys["y"][nl + part[hp]] + rng.normal(0, 1.5, int(hp.sum()))
        m["scale_level_r"][li[hp]] = F.keys["octave"][nl + part[hp]]
        # right source: right view near it, left view near its partner (or random)
        ri = cp[~left]
        rs = src[~left]
        m["proj_xr"][ri] = F.keys["x"][rs] + rng.normal(0, 1.5, len(ri))
        m["proj_yr"][ri] = F.keys["y"][rs] + rng.normal(0, 1.5, len(ri))
        m["scale_level_r"][ri] = F.keys["octave"][rs]
        part = F.r2l[rs - nl]
        hp = part >= 0
        m["proj_x"][ri[hp]] = F.keys["x"][part[hp]] + rng.normal(0, 1.5, int(hp.sum()))
        m["proj_y"][ri[hp]] = F.keys["y"][part[hp]] + rng.normal(0, 1.5, int(hp.sum()))
        m["scale_level"][ri[hp]] = F.keys["octave"][part[hp]]
    return m


def synth_proj_points_two(rng, F: MatchFrame, n: int, copy_frac: float = 0.8, flip_p: float = 0.05,
                          rot: float = 15.0):
    """Last-frame points for a two-camera current frame: (records, right_uv [n, 2]). Copies of a
    left feature land near it (and near its right partner in right_uv); the rest are random."""
    nl = F.nleft
    left = MatchFrame(F.keys[:nl], F.desc[:nl], F.bounds, F.scale_factors)
    p = synth_proj_points(rng, left, n, copy_frac=0.0, flip_p=flip_p, rot=rot)
    w, h = F.bounds[1], F.bounds[3]
    ruv = np.stack([rng.uniform(-20, w + 20, n), rng.uniform(-20, h + 20, n)], 1).astype(np.float32)
    if F.N:
        cp = np.nonzero(rng.random(n) < copy_frac)[0]
        src = rng.integers(0, F.N, len(cp))
        p["desc"][cp] = flip_bits(rng, F.desc[src], flip_p)
        lft = src < nl
        ls, rs = src[lft], src[~lft]
        lc, rc = cp[lft], cp[~lft]
        p["u"][lc] = F.keys["x"][ls] + rng.normal(0, 2.0, len(lc))
        p["v"][lc] = F.keys["y"][ls] + rng.normal(0, 2.0, len(lc))
        part = F.l2r[ls]
        hp = part >= 0
        ruv[lc[hp], 0] = F.keys["x"][nl + part[hp]] + rng.normal(0, 2.0, int(hp.sum()))
        ruv[lc[hp], 1] = F.keys["y"][nl + part[hp]] + rng.normal(0, 2.0, int(hp.sum()))
        ruv[rc, 0] = F.keys["x"][rs] + rng.normal(0, 2.0, len(rc))
        ruv[rc, 1] = F.keys["y"][rs] + rng.normal(0, 2.0, len(rc))
        part = F.r2l[rs - nl]
        hp = part >= 0
        p["u"][rc[hp]] = F.keys["x"][part[hp]] + rng.normal(0, 2.0, int(hp.sum()))
        p["v"][rc[hp]] = F.keys["y"][part[hp]] + rng.normal(0, 2.0, int(hp.sum()))
        p["octave"][cp] = np.clip(F.keys["octave"][src] + rng.integers(-1, 2, len(cp)), 0, len(F.scale_factors) - 1)
        outl = rng.random(len(cp)) < 0.15
        p["angle"][cp] = np.mod(np.where(outl, rng.uniform(0, 360, len(cp)),
                                         F.keys["angle"][src] + rot + rng.normal(0, 4, len(cp))), 360.0)
    return p, ruv


# ---- fisheye (KannalaBrandt8) frames: BASELINE config 4's TUM-VI rig (config/Stereo-Inertial/TUM-VI.yaml) ----
TUMVI_LEFT = (190.97847715128717, 190.9733070521226, 254.93170605935475, 256.8974428996504,
              (0.0034823894022493434, 0.0007150348452162257, -0.0020532361418706202, 0.00020293673591811182))
TUMVI_RIGHT = (190.44236969414825, 190.4344384721956, 252.59949716835982, 254.91723064636983,
               (0.0034003170790442797, 0.001766278153469831, -0.00266312569781606, 0.0003299517423931039))
TUMVI_TLR = np.array([[0.999999445773493, 0.000791687752817, 0.000694034010224, 0.101063427414194],
                      [-0.000823363992158, 0.998899461915674, 0.046895490788700, 0.001946204678584],
                      [-0.000656143613644, -0.046896036240590, 0.998899560146304, 0.001015350132563],
                      [0.0, 0.0, 0.0, 1.0]])


def kb8_unproject(u, v, fx, fy, cx, cy, k):
    """Unit rays of pixels under the KannalaBrandt8 model (float64 Newton on theta; the generator
    only needs rays that land near the pixels, the parity tests project them back with the model)."""
    px, py = (np.asarray(u, np.float64) - cx) / fx, (np.asarray(v, np.float64) - cy) / fy
    rd = np.minimum(np.hypot(px, py), np.pi / 2)
    th = rd.copy()
    for _ in range(30):
        t2 = th * th
        f = th * (1 + k[0] * t2 + k[1] * t2 ** 2 + k[2] * t2 ** 3 + k[3] * t2 ** 4) - rd
        df = 1 + 3 * k[0] * t2 + 5 * k[1] * t2 ** 2 + 7 * k[2] * t2 ** 3 + 9 * k[3] * t2 ** 4
        th = th - f / df
    psi = np.arctan2(py, px)
    return np.stack([np.sin(th) * np.cos(psi), np.sin(th) * np.sin(psi), np.cos(th)], 1)


def synth_rig(cam: Camera, two: bool = True):
    """The TUM-VI KannalaBrandt8 pair as a StereoRig (mpCamera, mpCamera2, mTrl / mTlr, mRwc)."""
    from .matcher import CameraModel, StereoRig
    left = CameraModel.make("kb8", *TUMVI_LEFT[:4], TUMVI_LEFT[4])
    right = CameraModel.make("kb8", *TUMVI_RIGHT[:4], TUMVI_RIGHT[4]) if two else None
    return StereoRig.make(left, right, TUMVI_TLR, np.array(cam.Rcw[:], np.float32).reshape(3, 3))


def synth_local_map_3d_rig(rng, F: MatchFrame, cam: Camera, n: int, two: bool = True, copy_frac: float = 0.5,
                           flip_p: float = 0.05, nlevels: int = 8, scale_factor: float = 1.2) -> np.ndarray:
    """synth_local_map_3d for a fisheye frame: points along the KannalaBrandt8 rays of pixels near
    frame keypoints (left ones, and with two cameras right ones through Tlr) or anywhere around
    the image, at 0.3-30 m; the same share of behind-camera / out-of-range / grazing / bad / seen
    points."""
    R = np.array(cam.Rcw[:], np.float64).reshape(3, 3)
    t = np.array(cam.tcw[:], np.float64)
    w, h = F.bounds[1], F.bounds[3]
    u = rng.uniform(-40, w + 40, n)
    v = rng.uniform(-40, h + 40, n)
    lvl = rng.choice(nlevels, n, p=level_weights(nlevels))
    desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    side = np.zeros(n, bool)
    if F.N:
        cp = np.nonzero(rng.random(n) < copy_frac)[0]
        src = rng.integers(0, F.N, len(cp))
        u[cp] = F.keys["x"][src] + rng.normal(0, 1.0, len(cp))
        v[cp] = F.keys["y"][src] + rng.normal(0, 1.0, len(cp))
        lvl[cp] = F.keys["octave"][src]
        desc[cp] = flip_bits(rng, F.desc[src], flip_p)
        if two and F.nleft is not None:
            side[cp] = src >= F.nleft
    s = rng.uniform(0.3, 30.0, n)
    s[rng.random(n) < 0.02] *= -1.0
    rays = kb8_unproject(u, v, *TUMVI_LEFT[:4], TUMVI_LEFT[4])
    Pc = rays * s[:, None]
    if two and side.any():
        rr = kb8_unproject(u[side], v[side], *TUMVI_RIGHT[:4], TUMVI_RIGHT[4]) * s[side][:, None]
        Pc[side] = rr @ TUMVI_TLR[:3, :3].T + TUMVI_TLR[:3, 3]      # right camera -> left camera
    P = (Pc - t) @ R
    dist = np.linalg.norm(P - np.array(cam.Ow[:], np.float64), axis=1)
    max_d = dist * scale_factor ** (lvl - rng.uniform(0.1, 0.9, n))
    out = rng.random(n) < 0.08
    max_d[out] *= rng.choice([0.5, 2.5], int(out.sum()))
    min_d = max_d / scale_factor ** (nlevels - 1)
    view = P - np.array(cam.Ow[:], np.float64)
    view /= np.maximum(np.linalg.norm(view, axis=1, keepdims=True), 1e-9)
    nrm = view + rng.normal(0, 0.3, (n, 3))
    graze = rng.random(n) < 0.05
    nrm[graze] = -nrm[graze]
    nrm /= np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-9)
    m = np.zeros(n, MAP_POINT_3D_DTYPE)
    m["pos"] = P.astype(np.float32)
    m["normal"] = nrm.astype(np.float32)
    m["min_dist"] = min_d.astype(np.float32)
    m["max_dist"] = max_d.astype(np.float32)
    fl = np.zeros(n, np.int32)
    fl[rng.random(n) < 0.03] |= MP_BAD
    fl[rng.random(n) < 0.03] |= MP_SKIP
    m["flags"] = fl
    m["observations"] = np.where(rng.random(n) < 0.1, 0, rng.integers(1, 20, n))
    m["id"] = np.arange(n) + 30000
    m["desc"] = desc
    # the previous frame's mTrackDepth (a two-camera point seen only by the right camera keeps it,
    # and bFarPoints reads it): 0-20 m against the tests' thFarPoints of 10 m
    m["track_depth"] = rng.uniform(0.0, 20.0, n).astype(np.float32)
    return m


def synth_two_cam_kf_pair(rng, nl: int, nr: int, words: int, rot: float = 20.0, drop: float = 0.15):
    """Two KannalaBrandt8 stereo keyframes (keys = mvKeys ++ mvKeysRight, NLeft = nl) sharing a scene:
    KF2 a perturbed copy of KF1 (both sides), map-point handles with NULL / bad slots, and
    FeatureVectors over every descriptor row (left and right, as the reference's mFeatVec)."""
    K1 = synth_frame_two(rng, nl, nr)
    P, src = perturbed_frame(rng, MatchFrame(K1.keys, K1.desc, K1.bounds, K1.scale_factors), rot=rot, flip_p=0.05,
                             drop=drop)
    K2 = MatchFrame(P.keys, P.desc, K1.bounds, K1.scale_factors, None, K1.mbf, nleft=nl, l2r=K1.l2r, r2l=K1.r2l)
    mp1 = np.where(rng.random(K1.N) < 0.2, -1, np.arange(K1.N) + 10).astype(np.int32)
    mp2 = np.where(rng.random(K2.N) < 0.2, -1, np.arange(K2.N) + 5000).astype(np.int32)
    fv1, fv2 = synth_bow(rng, words, K1, K2, src)
    return K1, K2, mp1, mp2, fv1, fv2, src


def right_kf_camera(cam: Camera, rig) -> KFCamera:
    """KeyFrame::GetRightPose() = mTrl * mTcw and GetRightCameraCenter() for a KFCamera (float64
    composition rounded to float32, as the caller's Sophus pose holds it)."""
    R = np.array(cam.Rcw[:], np.float64).reshape(3, 3)
    t = np.array(cam.tcw[:], np.float64)
    Rrl = np.array(rig.Rrl[:], np.float64).reshape(3, 3)
    trl = np.array(rig.trl[:], np.float64)
    Rr, tr = Rrl @ R, Rrl @ t + trl
    k = KFCamera.make(Pose.se3(Rr, tr), *TUMVI_RIGHT[:4])
    return k


def left_kf_camera(cam: Camera) -> KFCamera:
    R = np.array(cam.Rcw[:], np.float64).reshape(3, 3)
    t = np.array(cam.tcw[:], np.float64)
    return KFCamera.make(Pose.se3(R, t), *TUMVI_LEFT[:4])


def synth_pose(rng, rot_deg=10.0, t_scale=0.5):
    """A random rotation (up to rot_deg about a random axis) and translation, as float64 (R, t)."""
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    ang = np.deg2rad(rng.uniform(-rot_deg, rot_deg))
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    R = np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K
    return R, rng.normal(scale=t_scale, size=3)


def synth_last_points(rng, F: MatchFrame, model, R, t, n: int, copy_frac: float = 0.8, flip_p: float = 0.05,
                      rot: float = 15.0, nlevels: int = 8) -> np.ndarray:
    """Last-frame points in the world for the device-projected motion-model search (LAST_POINT
    records): copies of the frame's (left) keypoints sit on the keypoint's ray under `model` (pinhole
    or KannalaBrandt8) at a random depth for the pose x_c = R x_w + t, with flipped descriptor bits,
    the keypoint's octave +-1 and its angle + rot; the rest are random points in front of the camera.
    Some are invalid (no point / outlier), a few behind the camera."""
    from .matcher import LAST_POINT_DTYPE, CameraModel
    p = np.zeros(n, LAST_POINT_DTYPE)
    nl = F.nleft if F.nleft is not None else F.N
    fx, fy, cx, cy = (float(v) for v in model.params[:4])
    w, h = F.bounds[1], F.bounds[3]
    u = rng.uniform(0, w, n)
    v = rng.uniform(0, h, n)
    p["desc"] = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    p["octave"] = rng.integers(0, nlevels, n)
    p["angle"] = rng.uniform(0, 360, n)
    if nl:
        cp = np.nonzero(rng.random(n) < copy_frac)[0]
        src = rng.integers(0, nl, len(cp))
        u[cp] = F.keys["x"][src] + rng.normal(0, 1.5, len(cp))
        v[cp] = F.keys["y"][src] + rng.normal(0, 1.5, len(cp))
        p["desc"][cp] = flip_bits(rng, F.desc[src], flip_p)
        p["octave"][cp] = np.clip(F.keys["octave"][src] + rng.integers(-1, 2, len(cp)), 0, nlevels - 1)
        p["angle"][cp] = np.mod(F.keys["angle"][src] + rot + rng.normal(0, 4, len(cp)), 360.0)
    if model.type == CameraModel.KANNALA_BRANDT8:
        rays = kb8_unproject(u, v, fx, fy, cx, cy, [float(k) for k in model.params[4:8]])
    else:
        rays = np.stack([(u - cx) / fx, (v - cy) / fy, np.ones(n)], 1)
    depth = rng.uniform(1.0, 12.0, n)
    depth[rng.random(n) < 0.02] *= -1.0   # behind the camera
    c = rays * depth[:, None]
    p["pos"] = ((c - np.asarray(t)[None, :]) @ np.asarray(R)).astype(np.float32)   # R^T (c - t)
    p["observations"] = np.where(rng.random(n) < 0.1, 0, rng.integers(1, 20, n))
    p["id"] = np.arange(n) + 5000
    p["valid"] = (rng.random(n) > 0.05).astype(np.int32)
    return p

