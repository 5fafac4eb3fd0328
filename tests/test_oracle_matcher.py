"""CPU checks of the ORBmatcher oracle (oracle/orb_oracle_match.cpp) against an independent
pure-Python literal restatement of the reference loops (float32 arithmetic via numpy scalars) on
small seeded cases, plus properties of the synthetic workloads. No GPU needed."""
import math

import numpy as np
import pytest

from orb_slam3_ros_amd import synth_match as sm

f32 = np.float32


def _ham(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


class PyGrid:
    """Frame::AssignFeaturesToGrid + GetFeaturesInArea (Frame.cc:385-416, 657-723)."""

    def __init__(self, F):
        self.F = F
        self.invw = f32(64) / f32(f32(F.bounds[1]) - f32(F.bounds[0]))
        self.invh = f32(48) / f32(f32(F.bounds[3]) - f32(F.bounds[2]))
        self.cells = {}
        for i, k in enumerate(F.keys):
            px = int(round_half_away(f32(f32(k["x"] - f32(F.bounds[0])) * self.invw)))
            py = int(round_half_away(f32(f32(k["y"] - f32(F.bounds[2])) * self.invh)))
            if 0 <= px < 64 and 0 <= py < 48:
                self.cells.setdefault((px, py), []).append(i)

    def area(self, x, y, r, minL, maxL):
        F, x, y, r = self.F, f32(x), f32(y), f32(r)
        mnx, mny = f32(F.bounds[0]), f32(F.bounds[2])
        c0 = max(0, math.floor(f32(f32(f32(x - mnx) - r) * self.invw)))
        if c0 >= 64:
            return []
        c1 = min(63, math.ceil(f32(f32(f32(x - mnx) + r) * self.invw)))
        if c1 < 0:
            return []
        r0 = max(0, math.floor(f32(f32(f32(y - mny) - r) * self.invh)))
        if r0 >= 48:
            return []
        r1 = min(47, math.ceil(f32(f32(f32(y - mny) + r) * self.invh)))
        if r1 < 0:
            return []
        check = minL > 0 or maxL >= 0
        out = []
        for ix in range(c0, c1 + 1):
            for iy in range(r0, r1 + 1):
                for i in self.cells.get((ix, iy), []):
                    k = F.keys[i]
                    if check and (k["octave"] < minL or (maxL >= 0 and k["octave"] > maxL)):
                        continue
                    if abs(f32(k["x"] - x)) < r and abs(f32(k["y"] - y)) < r:
                        out.append(i)
        return out


def round_half_away(v):
    return math.floor(v + 0.5) if v >= 0 else -math.floor(-v + 0.5)


def py_sbp_local(F, mvp, obs, mps, th, nnratio):
    """ORBmatcher.cc:43-213 (pinhole path)."""
    g = PyGrid(F)
    obs = obs.copy()
    n = 0
    for mp in mps:
        if not (mp["flags"] & sm.MP_IN_VIEW) or (mp["flags"] & sm.MP_BAD):
            continue
        lvl = int(mp["scale_level"])
        r = f32(2.5) if float(mp["view_cos"]) > 0.998 else f32(4.0)
        if th != 1.0:
            r = f32(r * f32(th))
        R = f32(r * F.scale_factors[lvl])
        bd, bl, bd2, bl2, bi = 256, -1, 256, -1, -1
        for idx in g.area(mp["proj_x"], mp["proj_y"], R, lvl - 1, lvl):
            if mvp[idx] >= 0 and obs[idx] > 0:
                continue
            if F.uright is not None and F.uright[idx] > 0 and abs(f32(mp["proj_xr"] - F.uright[idx])) > R:
                continue
            d = _ham(mp["desc"], F.desc[idx])
            if d < bd:
                bd2, bd, bl2, bl, bi = bd, d, bl, int(F.keys[idx]["octave"]), idx
            elif d < bd2:
                bl2, bd2 = int(F.keys[idx]["octave"]), d
        if bd <= 100:
            if bl == bl2 and bd > f32(nnratio) * f32(bd2):
                continue
            mvp[bi] = mp["id"]
            obs[bi] = mp["observations"]
            n += 1
    return n


def py_search_for_init(F1, F2, prev, nnratio, window, check_ori):
    """ORBmatcher.cc:648-763."""
    g = PyGrid(F2)
    m12 = np.full(F1.N, -1, np.int32)
    md = [2**31 - 1] * F2.N
    m21 = [-1] * F2.N
    hist = [[] for _ in range(30)]
    n = 0
    for i1 in range(F1.N):
        if F1.keys[i1]["octave"] > 0:
            continue
        lvl = int(F1.keys[i1]["octave"])
        bd = bd2 = 2**31 - 1
        bi = -1
        for i2 in g.area(prev[i1, 0], prev[i1, 1], window, lvl, lvl):
            d = _ham(F1.desc[i1], F2.desc[i2])
            if md[i2] <= d:
                continue
            if d < bd:
                bd2, bd, bi = bd, d, i2
            elif d < bd2:
                bd2 = d
        if bd <= 50 and bd < f32(bd2) * f32(nnratio):
            if m21[bi] >= 0:
                m12[m21[bi]] = -1
                n -= 1
            m12[i1], m21[bi], md[bi] = bi, i1, bd
            n += 1
            if check_ori:
                rot = f32(F1.keys[i1]["angle"] - F2.keys[bi]["angle"])
                if rot < 0:
                    rot = f32(rot + f32(360))
                b = int(round_half_away(f32(rot * f32(f32(1) / f32(30)))))
                hist[0 if b == 30 else b].append(i1)
    if check_ori:
        sizes = [len(h) for h in hist]
        m1 = m2 = m3 = 0
        i1_ = i2_ = i3_ = -1
        for i, s in enumerate(sizes):
            if s > m1:
                m3, m2, m1, i3_, i2_, i1_ = m2, m1, s, i2_, i1_, i
            elif s > m2:
                m3, m2, i3_, i2_ = m2, s, i2_, i
            elif s > m3:
                m3, i3_ = s, i
        if m2 < 0.1 * m1:
            i2_ = i3_ = -1
        elif m3 < 0.1 * m1:
            i3_ = -1
        for i in range(30):
            if i in (i1_, i2_, i3_):
                continue
            for j in hist[i]:
                if m12[j] >= 0:
                    m12[j] = -1
                    n -= 1
    for i in range(F1.N):
        if m12[i] >= 0:
            prev[i] = (F2.keys[m12[i]]["x"], F2.keys[m12[i]]["y"])
    return n, m12


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_oracle_sbp_local_vs_python(oracle_lib, seed):
    rng = np.random.default_rng(seed)
    F = sm.synth_frame(rng, 150, w=200, h=150)
    mps = sm.synth_local_map(rng, F, 600, copy_frac=0.7, flip_p=0.03)
    mvp0, obs = sm.initial_slots(rng, F.N, 0.3)
    for th in (1, 3):
        a, b = mvp0.copy(), mvp0.copy()
        na = oracle_lib.OracleMatcher(0.8).sbp_local(F, a, obs, mps, th)
        nb = py_sbp_local(F, b, obs, mps, th, 0.8)
        assert na == nb and na > 0
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("seed", [3, 4])
def test_oracle_search_for_init_vs_python(oracle_lib, seed):
    rng = np.random.default_rng(seed)
    F1 = sm.synth_frame(rng, 300, w=200, h=150, stereo=False)
    F1.keys["octave"][rng.random(F1.N) < 0.6] = 0
    F2, _ = sm.perturbed_frame(rng, F1, shift=(2.0, 1.0), flip_p=0.04)
    prev = np.stack([F1.keys["x"], F1.keys["y"]], 1).astype(np.float32)
    pa, pb = prev.copy(), prev.copy()
    ma = np.zeros(F1.N, np.int32)
    na = oracle_lib.OracleMatcher(0.9, True).search_for_init(F1, F2, pa, ma, 20)
    nb, mb = py_search_for_init(F1, F2, pb, 0.9, 20, True)
    assert na == nb and na > 0
    np.testing.assert_array_equal(ma, mb)
    np.testing.assert_array_equal(pa, pb)


def test_oracle_knn_vs_numpy(oracle_lib):
    rng = np.random.default_rng(9)
    L = rng.integers(0, 256, (60, 32), dtype=np.uint8)
    R = rng.integers(0, 256, (80, 32), dtype=np.uint8)
    L[:30] = sm.flip_bits(rng, R[:30], 0.05)
    D = np.unpackbits(L[:, None, :] ^ R[None, :, :], axis=2).sum(2)
    g, t, d = oracle_lib.stereo_knn_ratio(L, R)
    for i in range(len(L)):
        order = np.argsort(D[i], kind="stable")
        d0, d1 = D[i, order[0]], D[i, order[1]]
        ok = d0 < d1 * 0.7
        assert t[i] == (order[0] if ok else -1)
        assert d[i] == (d0 if ok else -1)
    assert g == (t >= 0).sum() >= 25


def test_feature_vector_layout():
    fv = sm.FeatureVector({10: [3, 1], 2: [0], 7: []})
    assert fv.node_ids.tolist() == [2, 7, 10]
    assert fv.offsets.tolist() == [0, 1, 1, 3]
    assert fv.indices.tolist() == [0, 3, 1]


def test_record_layouts():
    import ctypes
    from orb_slam3_ros_amd.matcher import CFeatureVector, CFrame
    assert sm.MAP_POINT_DTYPE.itemsize == 80 and sm.PROJ_POINT_DTYPE.itemsize == 64
    assert ctypes.sizeof(CFrame) == 104 and CFrame.mbf.offset == 64
    assert CFrame.two_cams.offset == 68 and CFrame.nleft.offset == 72 and CFrame.l2r.offset == 80
    assert CFrame.device.offset == 96
    assert sm.MAP_POINT_DTYPE.fields["proj_yr"][1] == 36 and sm.MAP_POINT_DTYPE.fields["scale_level_r"][1] == 44
    assert ctypes.sizeof(CFeatureVector) == 32


def test_frame_layout_matches_header(tmp_path):
    """struct orbfe_frame as the C compiler lays it out (include/orbfe.h) == the ctypes mirror."""
    import ctypes
    import os
    import shutil
    import subprocess
    from orb_slam3_ros_amd.matcher import CFrame
    if shutil.which("gcc") is None:
        pytest.skip("needs gcc")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = tmp_path / "lay.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "orbfe.h"\nint main(void){printf("%zu %zu %zu",'
                   ' sizeof(orbfe_frame), offsetof(orbfe_frame, device), offsetof(orbfe_frame, r2l));return 0;}\n')
    exe = tmp_path / "lay"
    subprocess.run(["gcc", "-I", os.path.join(root, "include"), "-o", str(exe), str(src)], check=True)
    size, dev, r2l = map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split())
    assert (size, dev, r2l) == (ctypes.sizeof(CFrame), CFrame.device.offset, CFrame.r2l.offset)


def _golden_cases():
    import importlib.util
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    spec = importlib.util.spec_from_file_location("make_matcher_golden",
                                                  os.path.join(here, "golden", "make_matcher_golden.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    gold = np.load(os.path.join(here, "golden", "matcher_golden.npz"), allow_pickle=False)
    return mod, gold


def test_oracle_matcher_golden(oracle_lib):
    """The oracle reproduces the committed per-query fixtures (regression pin)."""
    mod, gold = _golden_cases()
    for name, kind, d in mod.cases():
        assert np.array_equal(mod.input_digest(kind, d), gold[name + "_in"]), f"{name}: generator drifted"
        res = mod.run(oracle_lib.OracleMatcher, kind, d)
        assert res[0] == int(gold[name + "_n"][0]), name
        for i, a in enumerate(res[1:]):
            assert np.array_equal(np.asarray(a), gold[f"{name}_out{i}"]), f"{name} output {i}"


def py_is_in_frustum(F, cam, pts):
    """Frame::isInFrustum (Frame.cc:512-570) + PredictScale (MapPoint.cc:531-546), float32 scalars."""
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    libm.logf.restype = ctypes.c_float
    libm.logf.argtypes = [ctypes.c_float]
    R = np.array(cam.Rcw[:], np.float32).reshape(3, 3)
    t = np.array(cam.tcw[:], np.float32)
    Ow = np.array(cam.Ow[:], np.float32)
    res = []
    for p in pts:
        if p["flags"] & (sm.MP_SKIP | sm.MP_BAD):
            res.append(None)
            continue
        P = p["pos"].astype(np.float32)
        # Eigen 3.3 fixed-size 3-term sums: a + (b + c) (redux_novec_unroller)
        Pc = [f32(f32(R[i, 0] * P[0]) + f32(f32(R[i, 1] * P[1]) + f32(R[i, 2] * P[2]))) + t[i] for i in range(3)]
        Pc = [f32(x) for x in Pc]
        Pc_dist = f32(np.sqrt(f32(f32(Pc[0] * Pc[0]) + f32(f32(Pc[1] * Pc[1]) + f32(Pc[2] * Pc[2])))))
        if Pc[2] < 0:
            res.append(None)
            continue
        invz = f32(f32(1) / Pc[2])
        u = f32(f32(f32(f32(cam.fx) * Pc[0]) / Pc[2]) + f32(cam.cx))
        v = f32(f32(f32(f32(cam.fy) * Pc[1]) / Pc[2]) + f32(cam.cy))
        if u < F.bounds[0] or u > F.bounds[1] or v < F.bounds[2] or v > F.bounds[3]:
            res.append(None)
            continue
        PO = [f32(P[i] - Ow[i]) for i in range(3)]
        dist = f32(np.sqrt(f32(f32(PO[0] * PO[0]) + f32(f32(PO[1] * PO[1]) + f32(PO[2] * PO[2])))))
        if dist < f32(f32(0.8) * p["min_dist"]) or dist > f32(f32(1.2) * p["max_dist"]):
            res.append(None)
            continue
        nrm = p["normal"]
        vc = f32(f32(f32(PO[0] * nrm[0]) + f32(f32(PO[1] * nrm[1]) + f32(PO[2] * nrm[2]))) / dist)
        if vc < f32(cam.view_cos_limit):
            res.append(None)
            continue
        ratio = f32(p["max_dist"] / dist)
        lv = int(math.ceil(f32(f32(libm.logf(float(ratio))) / f32(cam.log_scale_factor))))
        lv = min(max(lv, 0), len(F.scale_factors) - 1)
        res.append((u, v, f32(u - f32(f32(F.mbf) * invz)), Pc_dist, vc, lv))
    return res


@pytest.mark.parametrize("seed", [0, 1])
def test_oracle_frustum_vs_python(oracle_lib, seed):
    rng = np.random.default_rng(seed)
    F = sm.synth_frame(rng, 300)
    cam = sm.synth_camera(rng)
    pts = sm.synth_local_map_3d(rng, F, cam, 400)
    n, tr = oracle_lib.is_in_frustum(F, cam, pts)
    ref = py_is_in_frustum(F, cam, pts)
    assert n == sum(r is not None for r in ref) and n > 100
    for i, r in enumerate(ref):
        inv = bool(tr["flags"][i] & sm.MP_IN_VIEW)
        assert inv == (r is not None), i
        if r is not None:
            got = (tr["proj_x"][i], tr["proj_y"][i], tr["proj_xr"][i], tr["depth"][i], tr["view_cos"][i],
                   int(tr["scale_level"][i]))
            assert [np.float32(a).tobytes() for a in got[:5]] == [np.float32(b).tobytes() for b in r[:5]], i
            assert got[5] == r[5], i


def _py_three_maxima(hist):
    max1 = max2 = max3 = 0
    i1 = i2 = i3 = -1
    for i, c in enumerate(hist):
        if c > max1:
            max3, max2, max1, i3, i2, i1 = max2, max1, c, i2, i1, i
        elif c > max2:
            max3, max2, i3, i2 = max2, c, i2, i
        elif c > max3:
            max3, i3 = c, i
    if max2 < f32(0.1) * f32(max1):
        i2 = i3 = -1
    elif max3 < f32(0.1) * f32(max1):
        i3 = -1
    return {i1, i2, i3}


def _py_rot_bin(a1, a2):
    rot = f32(f32(a1) - f32(a2))
    if rot < 0.0:
        rot = f32(rot + f32(360.0))
    b = int(round_half_away(f32(rot * f32(f32(1.0) / f32(30)))))
    return 0 if b == 30 else b


def py_search_by_bow_kf(k1, d1, mp1, fv1, k2, d2, mp2, fv2, nnratio, check_ori):
    """ORBmatcher::SearchByBoW(KF, KF) (ORBmatcher.cc:765-903), literal."""
    out = np.full(len(k1), -1, np.int32)
    matched2 = np.zeros(len(k2), bool)
    nodes2 = {int(n): fv2.indices[fv2.offsets[j]:fv2.offsets[j + 1]] for j, n in enumerate(fv2.node_ids)}
    hist = [[] for _ in range(30)]
    n = 0
    for a, node in enumerate(fv1.node_ids):
        if int(node) not in nodes2:
            continue
        for i1 in fv1.indices[fv1.offsets[a]:fv1.offsets[a + 1]]:
            if mp1[i1] < 0:
                continue
            b1, bi, b2 = 256, -1, 256
            for i2 in nodes2[int(node)]:
                if matched2[i2] or mp2[i2] < 0:
                    continue
                d = _ham(d1[i1], d2[i2])
                if d < b1:
                    b2, b1, bi = b1, d, int(i2)
                elif d < b2:
                    b2 = d
            if b1 < 50 and f32(b1) < f32(f32(nnratio) * f32(b2)):
                out[i1] = mp2[bi]
                matched2[bi] = True
                if check_ori:
                    hist[_py_rot_bin(k1[i1]["angle"], k2[bi]["angle"])].append(int(i1))
                n += 1
    if check_ori:
        keep = _py_three_maxima([len(h) for h in hist])
        for i, h in enumerate(hist):
            if i not in keep:
                for j in h:
                    out[j] = -1
                    n -= 1
    return n, out


def py_distinctive(sets):
    """MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:329-403)."""
    best = []
    for d in sets:
        N = len(d)
        if N == 0:
            best.append(-1)
            continue
        D = np.unpackbits(d[:, None, :] ^ d[None, :, :], axis=2).sum(2)
        med = [int(np.sort(D[i])[int(0.5 * (N - 1))]) for i in range(N)]
        best.append(int(np.argmin(med)))   # argmin = first minimum
    return np.array(best, np.int32)


@pytest.mark.parametrize("seed,check_ori", [(0, True), (1, False), (2, True)])
def test_oracle_bow_kf_vs_python(oracle_lib, seed, check_ori):
    rng = np.random.default_rng(seed)
    K1, K2, mp1, mp2, fv1, fv2 = sm.synth_kf_pair(rng, 250, 40)
    no, oo = oracle_lib.OracleMatcher(0.75, check_ori).search_by_bow_kf(K1.keys, K1.desc, mp1, fv1, K2.keys,
                                                                          K2.desc, mp2, fv2)
    np_, op = py_search_by_bow_kf(K1.keys, K1.desc, mp1, fv1, K2.keys, K2.desc, mp2, fv2, 0.75, check_ori)
    assert no == np_ and no > 0
    np.testing.assert_array_equal(oo, op)
    assert no == (oo >= 0).sum()


def test_oracle_distinctive_vs_python(oracle_lib):
    rng = np.random.default_rng(5)
    sets = sm.synth_distinctive_sets(rng, [0, 1, 2, 3, 4, 7, 30, 64, 65, 130])
    offs = np.zeros(len(sets) + 1, np.int32)
    offs[1:] = np.cumsum([len(d) for d in sets])
    got = oracle_lib.distinctive_descriptors(np.concatenate(sets), offs)
    np.testing.assert_array_equal(got, py_distinctive(sets))
    assert got[0] == -1 and got[1] == 0


# ---- back-end projections: literal float32 restatements ----
def _py_pose_apply(P, p):
    vx, vy, vz, w = (f32(v) for v in P.q)
    t = [f32(v) for v in P.t]
    p = [f32(v) for v in p]
    uv = [f32(vy * p[2] - vz * p[1]), f32(vz * p[0] - vx * p[2]), f32(vx * p[1] - vy * p[0])]
    uv = [f32(u + u) for u in uv]
    c = [f32(vy * uv[2] - vz * uv[1]), f32(vz * uv[0] - vx * uv[2]), f32(vx * uv[1] - vy * uv[0])]
    if P.kind == 1:
        sc = f32(f32(vx * vx + vz * vz) + f32(vy * vy + w * w))
        return [f32(f32(sc * p[k] + f32(w * uv[k] + c[k])) + t[k]) for k in range(3)]
    return [f32(f32(f32(p[k] + w * uv[k]) + c[k]) + t[k]) for k in range(3)]


def _py_predict(max_dist, dist, logsf, nlevels):
    ratio = f32(f32(max_dist) / f32(dist))
    n = int(math.ceil(f32(f32(np.log(ratio)) / f32(logsf))))   # numpy float32 log (parity of logf is tested natively)
    return min(max(n, 0), nlevels - 1)


def _py_in_image(F, x, y):
    return F.bounds[0] <= x < F.bounds[1] and F.bounds[2] <= y < F.bounds[3]


def py_fuse(KF, cam, pts, th, sim3):
    g = PyGrid(KF)
    inv = (f32(1.0) / (KF.scale_factors * KF.scale_factors)).astype(np.float32)
    bi = np.full(len(pts), -1, np.int32)
    bd = np.full(len(pts), -1, np.int32)
    for i, mp in enumerate(pts):
        if mp["flags"] & 6 or mp["id"] < 0:
            continue
        pc = _py_pose_apply(cam.Tcw, mp["pos"])
        if pc[2] < 0:
            continue
        invz = f32(f32(1) / pc[2])
        u = f32(f32(f32(cam.fx) * pc[0]) / pc[2] + f32(cam.cx))
        v = f32(f32(f32(cam.fy) * pc[1]) / pc[2] + f32(cam.cy))
        if not _py_in_image(KF, u, v):
            continue
        ur = f32(u - f32(KF.mbf) * invz)
        PO = [f32(mp["pos"][k] - f32(cam.Ow[k])) for k in range(3)]
        d = f32(np.sqrt(f32(f32(PO[0] * PO[0]) + f32(f32(PO[1] * PO[1]) + f32(PO[2] * PO[2])))))
        if d < f32(f32(0.8) * mp["min_dist"]) or d > f32(f32(1.2) * mp["max_dist"]):
            continue
        dot = f32(f32(PO[0] * mp["normal"][0]) + f32(f32(PO[1] * mp["normal"][1]) + f32(PO[2] * mp["normal"][2])))
        if float(dot) < 0.5 * float(d):
            continue
        lvl = _py_predict(mp["max_dist"], d, cam.log_scale_factor, len(KF.scale_factors))
        r = f32(f32(th) * KF.scale_factors[lvl])
        best, bidx = (2 ** 31 - 1 if sim3 else 256), -1
        for idx in g.area(u, v, r, -1, -1):
            kp = KF.keys[idx]
            if kp["octave"] < lvl - 1 or kp["octave"] > lvl:
                continue
            if not sim3:
                ex, ey = f32(u - kp["x"]), f32(v - kp["y"])
                if KF.uright is not None and KF.uright[idx] >= 0:
                    er = f32(ur - KF.uright[idx])
                    e2 = f32(f32(ex * ex + ey * ey) + er * er)
                    if float(f32(e2 * inv[kp["octave"]])) > 7.8:
                        continue
                else:
                    e2 = f32(ex * ex + ey * ey)
                    if float(f32(e2 * inv[kp["octave"]])) > 5.99:
                        continue
            dd = _ham(mp["desc"], KF.desc[idx])
            if dd < best:
                best, bidx = dd, idx
        if bidx >= 0:
            bd[i] = best
        if best <= 50:
            bi[i] = bidx
    return int((bi >= 0).sum()), bi, bd


@pytest.mark.parametrize("sim3", [0, 1])
def test_oracle_fuse_vs_python(oracle_lib, sim3):
    rng = np.random.default_rng(31 + sim3)
    KF, cam, pts = sm.synth_fuse_scene(rng, 300, 500, dup=2)
    n, bi, bd = oracle_lib.OracleMatcher().fuse(KF, cam, pts, 3.0, sim3=sim3)
    n2, bi2, bd2 = py_fuse(KF, cam, pts, 3.0, sim3)
    assert n == n2 and n > 20
    np.testing.assert_array_equal(bi, bi2)
    np.testing.assert_array_equal(bd, bd2)


def py_search_by_sim3(K1, K2, p1, p2, c1, c2, S12, S21, th, m12):
    def side(B, ptsA, already, TAw, SBA, logsfB):
        g = PyGrid(B)
        vn = np.full(len(ptsA), -1, np.int64)
        for i, mp in enumerate(ptsA):
            if mp["id"] < 0 or already[i] or mp["flags"] & 2:
                continue
            pB = _py_pose_apply(SBA, _py_pose_apply(TAw, mp["pos"]))
            if pB[2] < 0:
                continue
            invz = f32(1.0 / float(pB[2]))
            u = f32(f32(c1.fx) * f32(pB[0] * invz) + f32(c1.cx))
            v = f32(f32(c1.fy) * f32(pB[1] * invz) + f32(c1.cy))
            if not _py_in_image(B, u, v):
                continue
            d = f32(np.sqrt(f32(f32(pB[0] * pB[0]) + f32(f32(pB[1] * pB[1]) + f32(pB[2] * pB[2])))))
            if d < f32(f32(0.8) * mp["min_dist"]) or d > f32(f32(1.2) * mp["max_dist"]):
                continue
            lvl = _py_predict(mp["max_dist"], d, logsfB, len(B.scale_factors))
            r = f32(f32(th) * B.scale_factors[lvl])
            best, bidx = 2 ** 31 - 1, -1
            for idx in g.area(u, v, r, -1, -1):
                o = B.keys[idx]["octave"]
                if o < lvl - 1 or o > lvl:
                    continue
                dd = _ham(mp["desc"], B.desc[idx])
                if dd < best:
                    best, bidx = dd, idx
            if best <= 100:
                vn[i] = bidx
        return vn
    a1 = m12 >= 0
    vn1 = side(K2, p1, a1, c1.Tcw, S21, c2.log_scale_factor)
    vn2 = side(K1, p2, np.zeros(K2.N, bool), c2.Tcw, S12, c1.log_scale_factor)
    out = m12.copy()
    n = 0
    for i1 in range(K1.N):
        j = vn1[i1]
        if j >= 0 and vn2[j] == i1:
            out[i1] = p2[j]["id"]
            n += 1
    return n, out


@pytest.mark.parametrize("scale", [1.0, 1.3])
def test_oracle_search_by_sim3_vs_python(oracle_lib, scale):
    rng = np.random.default_rng(40)
    K1, K2, p1, p2, c1, c2, S12, S21, _ = sm.synth_sim3_pair(rng, 250, scale=scale)
    m = np.full(K1.N, -1, np.int32)
    m[:10] = 7   # initial matches (no KF2 index given)
    mo = m.copy()
    n = oracle_lib.OracleMatcher().search_by_sim3(K1, K2, p1, p2, c1, c2, S12, S21, 7.5, mo)
    n2, mp = py_search_by_sim3(K1, K2, p1, p2, c1, c2, S12, S21, 7.5, m)
    assert n == n2
    np.testing.assert_array_equal(mo, mp)
    if scale == 1.0:
        assert n > 50


def _libm():
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    for fn in ("logf", "cosf", "sinf"):
        getattr(libm, fn).restype = ctypes.c_float
        getattr(libm, fn).argtypes = [ctypes.c_float]
    libm.atan2f.restype = ctypes.c_float
    libm.atan2f.argtypes = [ctypes.c_float, ctypes.c_float]
    return libm


def _py_kb8(m, x, y, z, libm):
    """KannalaBrandt8::project (KannalaBrandt8.cpp:67-82), float32 scalars in source order."""
    p = [f32(v) for v in m.params]
    theta = f32(libm.atan2f(float(np.sqrt(f32(f32(x * x) + f32(y * y)))), float(z)))
    psi = f32(libm.atan2f(float(y), float(x)))
    t2 = f32(theta * theta)
    t3 = f32(theta * t2)
    t5 = f32(t3 * t2)
    t7 = f32(t5 * t2)
    t9 = f32(t7 * t2)
    r = f32(f32(f32(f32(theta + f32(p[4] * t3)) + f32(p[5] * t5)) + f32(p[6] * t7)) + f32(p[7] * t9))
    return (f32(f32(f32(p[0] * r) * f32(libm.cosf(float(psi)))) + p[2]),
            f32(f32(f32(p[1] * r) * f32(libm.sinf(float(psi)))) + p[3]))


def _py_view(F, cam, R, t, Ow, model, p, libm):
    """isInFrustumChecks for one view (Frame.cc:1168-1242) with Eigen 3.3's a + (b + c) sums;
    returns (u, v, level, viewcos, depth) or None."""
    P = p["pos"].astype(np.float32)
    Pc = [f32(f32(f32(R[i, 0] * P[0]) + f32(f32(R[i, 1] * P[1]) + f32(R[i, 2] * P[2]))) + t[i]) for i in range(3)]
    depth = f32(np.sqrt(f32(f32(Pc[0] * Pc[0]) + f32(f32(Pc[1] * Pc[1]) + f32(Pc[2] * Pc[2])))))
    if Pc[2] < 0:
        return None
    u, v = _py_kb8(model, Pc[0], Pc[1], Pc[2], libm)
    if u < F.bounds[0] or u > F.bounds[1] or v < F.bounds[2] or v > F.bounds[3]:
        return None
    PO = [f32(P[i] - Ow[i]) for i in range(3)]
    dist = f32(np.sqrt(f32(f32(PO[0] * PO[0]) + f32(f32(PO[1] * PO[1]) + f32(PO[2] * PO[2])))))
    if dist < f32(f32(0.8) * p["min_dist"]) or dist > f32(f32(1.2) * p["max_dist"]):
        return None
    nrm = p["normal"]
    vc = f32(f32(f32(PO[0] * nrm[0]) + f32(f32(PO[1] * nrm[1]) + f32(PO[2] * nrm[2]))) / dist)
    if vc < f32(cam.view_cos_limit):
        return None
    lv = int(math.ceil(f32(f32(libm.logf(float(f32(p["max_dist"] / dist)))) / f32(cam.log_scale_factor))))
    return u, v, min(max(lv, 0), len(F.scale_factors) - 1), vc, depth


@pytest.mark.parametrize("two", [False, True])
def test_oracle_frustum_rig_vs_python(oracle_lib, two):
    """Frame::isInFrustum with KannalaBrandt8 cameras (Frame.cc:512-586, 1168-1242): the C++ oracle
    against a float32 Python restatement, a monocular fisheye frame and a two-camera frame."""
    libm = _libm()
    rng = np.random.default_rng(40 + two)
    F = sm.synth_frame_two(rng, 300, 280) if two else sm.synth_frame(rng, 300, 512, 512, stereo=False)
    cam = sm.synth_camera(rng, rot_deg=20.0)
    rig = sm.synth_rig(cam, two)
    pts = sm.synth_local_map_3d_rig(rng, F, cam, 600, two=two)
    n, tr = oracle_lib.is_in_frustum(F, cam, pts, rig)
    R = np.array(cam.Rcw[:], np.float32).reshape(3, 3)
    t = np.array(cam.tcw[:], np.float32)
    Ow = np.array(cam.Ow[:], np.float32)
    # right view: mR = Rrl * mRcw, mt = Rrl * mtcw + trl, twc = mRwc * tlr + mOw (a + (b + c) sums)
    A = np.array(rig.Rrl[:], np.float32).reshape(3, 3)
    Rwc = np.array(rig.Rwc[:], np.float32).reshape(3, 3)
    s3 = lambda a, b, c: f32(f32(a) + f32(f32(b) + f32(c)))   # noqa: E731
    R2 = np.array([[s3(A[i, 0] * R[0, j], A[i, 1] * R[1, j], A[i, 2] * R[2, j]) for j in range(3)] for i in range(3)],
                  np.float32)
    t2 = np.array([f32(s3(A[i, 0] * t[0], A[i, 1] * t[1], A[i, 2] * t[2]) + f32(rig.trl[i])) for i in range(3)],
                  np.float32)
    tl = np.array(rig.tlr[:], np.float32)
    Ow2 = np.array([f32(s3(Rwc[i, 0] * tl[0], Rwc[i, 1] * tl[1], Rwc[i, 2] * tl[2]) + Ow[i]) for i in range(3)],
                   np.float32)
    count = nr = 0
    for i, p in enumerate(pts):
        if p["flags"] & (sm.MP_SKIP | sm.MP_BAD):
            assert not tr["flags"][i] & (sm.MP_IN_VIEW | sm.MP_IN_VIEW_R)
            continue
        lv = _py_view(F, cam, R, t, Ow, rig.left, p, libm)
        rv = _py_view(F, cam, R2, t2, Ow2, rig.right, p, libm) if two else None
        assert bool(tr["flags"][i] & sm.MP_IN_VIEW) == (lv is not None), i
        assert bool(tr["flags"][i] & sm.MP_IN_VIEW_R) == (rv is not None), i
        if lv is not None:
            got = (tr["proj_x"][i], tr["proj_y"][i], int(tr["scale_level"][i]), tr["view_cos"][i], tr["depth"][i])
            assert [np.float32(a).tobytes() for a in (got[0], got[1], got[3], got[4])] == \
                [np.float32(b).tobytes() for b in (lv[0], lv[1], lv[3], lv[4])], i
            assert got[2] == lv[2], i
        if rv is not None:
            nr += 1
            got = (tr["proj_xr"][i], tr["proj_yr"][i], int(tr["scale_level_r"][i]), tr["view_cos_r"][i])
            assert [np.float32(a).tobytes() for a in (got[0], got[1], got[3])] == \
                [np.float32(b).tobytes() for b in (rv[0], rv[1], rv[3])], i
            assert got[2] == rv[2], i
        count += (lv is not None) or (rv is not None)
    assert n == count and n > 150
    assert nr > 100 or not two


@pytest.mark.parametrize("seed", [31, 32])
def test_oracle_lastframe_pose_identity(oracle_lib, seed):
    """The oracle's device-projection restatement (oro_sbp_lastframe_pose) with the identity rotation
    and a pinhole camera, where Sophus' action reduces to x + t exactly: the projected records rebuilt
    in numpy float32 (u = fx * x / z + cx, invzc = float(1.0 / double(z))) give the same search
    through the host-projected entry point, slots included."""
    from orb_slam3_ros_amd.matcher import PROJ_POINT_DTYPE, CameraModel, Pose
    rng = np.random.default_rng(seed)
    F = sm.synth_frame(rng, 800)
    model = CameraModel.make("pinhole", 458.654, 457.296, 367.215, 248.375)
    t = rng.normal(scale=0.3, size=3).astype(np.float32)
    pts = sm.synth_last_points(rng, F, model, np.eye(3), t.astype(np.float64), 900)
    Tcw = Pose.se3(np.eye(3), t)
    assert list(Tcw.q) == [0.0, 0.0, 0.0, 1.0]
    c = (pts["pos"] + t[None, :]).astype(np.float32)
    rec = np.zeros(len(pts), PROJ_POINT_DTYPE)
    for f in ("octave", "angle", "observations", "id", "valid", "desc"):
        rec[f] = pts[f]
    with np.errstate(divide="ignore", invalid="ignore"):
        rec["invzc"] = (1.0 / c[:, 2].astype(np.float64)).astype(np.float32)
        fx, fy, cx, cy = (np.float32(v) for v in model.params[:4])
        rec["u"] = np.where(rec["valid"] != 0, fx * c[:, 0] / c[:, 2] + cx, 0).astype(np.float32)
        rec["v"] = np.where(rec["valid"] != 0, fy * c[:, 1] / c[:, 2] + cy, 0).astype(np.float32)
    mvp0, obs = sm.initial_slots(rng, F.N, 0.2)
    om = oracle_lib.OracleMatcher(0.9, True)
    for th, fw, bw in [(7, False, False), (15, True, False)]:
        a, b = mvp0.copy(), mvp0.copy()
        na = om.sbp_lastframe_pose(F, a, obs, pts, Tcw, model, th, fw, bw)
        nb = om.sbp_lastframe(F, b, obs, rec, th, fw, bw)
        assert na == nb and na > 20
        np.testing.assert_array_equal(a, b)

