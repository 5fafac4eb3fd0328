"""GPU parity: the HIP ORBmatcher methods (through the C-ABI) against the CPU oracle's literal
sequential restatement (oracle/orb_oracle_match.cpp), on seeded synthetic frames / map points.
Match sets (every mvpMapPoints slot, vnMatches12, vbPrevMatched, SearchByBoW output) and
nmatches must be identical. Includes the BASELINE config-5 stress: 100k map points against a
1000- and a 5000-keypoint frame at th in {1, 3, 5, 15}, seed 12345.
Parity is "unpinned" w.r.t. the real reference (no buildable reference, no matcher fixtures in
it): the oracle is the restatement, see DESIGN.md.
"""
import numpy as np
import pytest

from orb_slam3_ros_amd import synth_match as sm
from orb_slam3_ros_amd.matcher import MatchFrame, ORBmatcher, stereo_knn_ratio

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def om(oracle_lib):
    return oracle_lib


def _local_case(seed, n_kp, n_mps, stereo=True, slots=0.1, copy_frac=0.3):
    rng = np.random.default_rng(seed)
    F = sm.synth_frame(rng, n_kp, stereo=stereo)
    mps = sm.synth_local_map(rng, F, n_mps, copy_frac=copy_frac)
    mvp, obs = sm.initial_slots(rng, n_kp, slots)
    return F, mps, mvp, obs


@pytest.mark.parametrize("th", [1, 3, 5, 15])
@pytest.mark.parametrize("n_kp", [1000, 5000])
def test_sbp_local_config5(gpu, om, th, n_kp):
    F, mps, mvp0, obs = _local_case(12345, n_kp, 100_000)
    m = ORBmatcher(0.8)
    mvp_g = mvp0.copy()
    ng = m.SearchByProjection(F, mvp_g, obs, mps, th)
    mvp_o = mvp0.copy()
    no = om.OracleMatcher(0.8).sbp_local(F, mvp_o, obs, mps, th)
    assert ng == no
    np.testing.assert_array_equal(mvp_g, mvp_o)
    assert no > 0


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("stereo,bfar,ratio", [(True, False, 0.8), (False, False, 0.8), (True, True, 0.6)])
def test_sbp_local_variants(gpu, om, seed, stereo, bfar, ratio):
    F, mps, mvp0, obs = _local_case(seed, 1200, 8000, stereo=stereo, slots=0.3, copy_frac=0.6)
    mvp_g, mvp_o = mvp0.copy(), mvp0.copy()
    ng = ORBmatcher(ratio).SearchByProjectionLocalMap(F, mvp_g, obs, mps, 1.0, bfar, 20.0)
    no = om.OracleMatcher(ratio).sbp_local(F, mvp_o, obs, mps, 1.0, bfar, 20.0)
    assert ng == no
    np.testing.assert_array_equal(mvp_g, mvp_o)


def test_sbp_local_dense_conflicts(gpu, om):
    """Many map points competing for few keypoints with Observations() == 0 slots: the ordered
    'later points see earlier assignments' chain is long here."""
    rng = np.random.default_rng(7)
    F = sm.synth_frame(rng, 300, w=120, h=90)
    mps = sm.synth_local_map(rng, F, 20000, copy_frac=0.9, flip_p=0.02)
    mps["observations"] = np.where(rng.random(len(mps)) < 0.5, 0, mps["observations"])
    mvp0 = np.full(F.N, -1, np.int32)
    obs = np.zeros(F.N, np.int32)
    for th in (1, 3, 15):
        a, b = mvp0.copy(), mvp0.copy()
        ng = ORBmatcher(0.8).SearchByProjectionLocalMap(F, a, obs, mps, th)
        no = om.OracleMatcher(0.8).sbp_local(F, b, obs, mps, th)
        assert ng == no
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("seed", [11, 12, 13, 14])
@pytest.mark.parametrize("mode", ["none", "forward", "backward"])
@pytest.mark.parametrize("check_ori", [True, False])
def test_sbp_lastframe(gpu, om, seed, mode, check_ori):
    rng = np.random.default_rng(seed)
    F = sm.synth_frame(rng, 1500, stereo=seed % 2 == 0)
    pts = sm.synth_proj_points(rng, F, 1400)
    mvp0, obs = sm.initial_slots(rng, F.N, 0.2)
    for th in (7, 15):
        a, b = mvp0.copy(), mvp0.copy()
        fw, bw = mode == "forward", mode == "backward"
        ng = ORBmatcher(0.9, check_ori).SearchByProjectionLastFrame(F, a, obs, pts, th, fw, bw)
        no = om.OracleMatcher(0.9, check_ori).sbp_lastframe(F, b, obs, pts, th, fw, bw)
        assert ng == no
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("seed", [21, 22, 23])
@pytest.mark.parametrize("check_ori", [True, False])
def test_sbp_keyframe(gpu, om, seed, check_ori):
    rng = np.random.default_rng(seed)
    F = sm.synth_frame(rng, 1000, stereo=False)
    pts = sm.synth_proj_points(rng, F, 1200, copy_frac=0.7)
    mvp0, _ = sm.initial_slots(rng, F.N, 0.25)
    for th, orbdist in ((10, 100), (3, 64)):
        a, b = mvp0.copy(), mvp0.copy()
        ng = ORBmatcher(0.9, check_ori).SearchByProjectionKeyFrame(F, a, pts, th, orbdist)
        no = om.OracleMatcher(0.9, check_ori).sbp_kf(F, b, pts, th, orbdist)
        assert ng == no
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("seed", [31, 32, 33, 34])
@pytest.mark.parametrize("window", [10, 100])
def test_search_for_initialization(gpu, om, seed, window):
    rng = np.random.default_rng(seed)
    F1 = sm.synth_frame(rng, 2000, stereo=False)
    F2, _ = sm.perturbed_frame(rng, F1, shift=(6.0, -4.0), jitter=2.0, rot=12.0, flip_p=0.06, drop=0.2)
    prev0 = np.stack([F1.keys["x"], F1.keys["y"]], 1).astype(np.float32)
    for check_ori in (True, False):
        pa, pb = prev0.copy(), prev0.copy()
        ma, mb = np.zeros(F1.N, np.int32), np.zeros(F1.N, np.int32)
        ng = ORBmatcher(0.9, check_ori).SearchForInitialization(F1, F2, pa, ma, window)
        no = om.OracleMatcher(0.9, check_ori).search_for_init(F1, F2, pb, mb, window)
        assert ng == no
        np.testing.assert_array_equal(ma, mb)
        np.testing.assert_array_equal(pa, pb)


def test_search_for_initialization_steals(gpu, om):
    """Dense clone clusters: many F1 features select the same F2 feature, so vnMatches21
    steals and vMatchedDistance updates chain through the query order."""
    rng = np.random.default_rng(5)
    F1 = sm.synth_frame(rng, 1500, w=160, h=120, stereo=False)
    base = F1.desc[:20]
    F1.desc[:] = sm.flip_bits(rng, base[rng.integers(0, 20, F1.N)], 0.03)
    F1.keys["octave"][:] = 0
    F2, _ = sm.perturbed_frame(rng, F1, shift=(1.0, 1.0), flip_p=0.03, drop=0.0)
    prev0 = np.stack([F1.keys["x"], F1.keys["y"]], 1).astype(np.float32)
    pa, pb = prev0.copy(), prev0.copy()
    ma, mb = np.zeros(F1.N, np.int32), np.zeros(F1.N, np.int32)
    ng = ORBmatcher(0.95, True).SearchForInitialization(F1, F2, pa, ma, 40)
    no = om.OracleMatcher(0.95, True).search_for_init(F1, F2, pb, mb, 40)
    assert ng == no
    np.testing.assert_array_equal(ma, mb)
    np.testing.assert_array_equal(pa, pb)


@pytest.mark.parametrize("seed", [41, 42, 43])
@pytest.mark.parametrize("check_ori", [True, False])
def test_search_by_bow(gpu, om, seed, check_ori):
    rng = np.random.default_rng(seed)
    KF = sm.synth_frame(rng, 1000, stereo=False)
    F, src = sm.perturbed_frame(rng, KF, rot=20.0, flip_p=0.05, drop=0.15)
    kf_mp = np.where(rng.random(KF.N) < 0.25, -1, np.arange(KF.N) + 100).astype(np.int32)
    for words in (50, 400):
        fk, ff = sm.synth_bow(rng, words, KF, F, src)
        ng, out_g = ORBmatcher(0.75, check_ori).SearchByBoW(KF.keys, KF.desc, kf_mp, fk, F, ff)
        no, out_o = om.OracleMatcher(0.75, check_ori).search_by_bow(KF.keys, KF.desc, kf_mp, fk, F, ff)
        assert ng == no
        np.testing.assert_array_equal(out_g, out_o)
        assert no > 0


@pytest.mark.parametrize("n_kf,n_f,words", [
    (1000, 1000, 1),      # one node: a 1000 x 1000 walk through the LDS form of k_bow_block
    (3000, 3000, 400),    # beyond k_bow_block's LDS (the multi-launch k_bow_nodes + k_bow_commit)
    (1200, 1100, 5000),   # mostly single-feature nodes, many without a partner node
])
def test_search_by_bow_sizes(gpu, om, n_kf, n_f, words):
    rng = np.random.default_rng(n_kf + 7 * words)
    KF = sm.synth_frame(rng, n_kf, stereo=False)
    F, src = sm.perturbed_frame(rng, KF, rot=20.0, flip_p=0.05, drop=0.15)
    F = MatchFrame(F.keys[:n_f].copy(), F.desc[:n_f].copy(), F.bounds, F.scale_factors)
    src = src[:n_f]
    kf_mp = np.where(rng.random(KF.N) < 0.25, -1, np.arange(KF.N) + 100).astype(np.int32)
    fk, ff = sm.synth_bow(rng, words, KF, F, src)
    for check_ori in (True, False):
        ng, out_g = ORBmatcher(0.75, check_ori).SearchByBoW(KF.keys, KF.desc, kf_mp, fk, F, ff)
        no, out_o = om.OracleMatcher(0.75, check_ori).search_by_bow(KF.keys, KF.desc, kf_mp, fk, F, ff)
        assert ng == no
        np.testing.assert_array_equal(out_g, out_o)


def test_search_for_initialization_5000(gpu, om):
    """The monocular initialiser's size (5 x nFeatures): one query row of 16 lanes per F1 feature."""
    rng = np.random.default_rng(4242)
    F1 = sm.synth_frame(rng, 5000, stereo=False)
    F2, _ = sm.perturbed_frame(rng, F1, shift=(6.0, -4.0), jitter=2.0, rot=12.0, flip_p=0.06, drop=0.2)
    prev0 = np.stack([F1.keys["x"], F1.keys["y"]], 1).astype(np.float32)
    pa, pb = prev0.copy(), prev0.copy()
    ma, mb = np.zeros(F1.N, np.int32), np.zeros(F1.N, np.int32)
    ng = ORBmatcher(0.9, True).SearchForInitialization(F1, F2, pa, ma, 100)
    no = om.OracleMatcher(0.9, True).search_for_init(F1, F2, pb, mb, 100)
    assert ng == no and no > 0
    np.testing.assert_array_equal(ma, mb)
    np.testing.assert_array_equal(pa, pb)


@pytest.mark.parametrize("nl,nr", [(1000, 1000), (1, 2), (333, 517), (700, 1)])
def test_stereo_knn_ratio(gpu, om, nl, nr):
    rng = np.random.default_rng(nl * 7 + nr)
    R = rng.integers(0, 256, (nr, 32), dtype=np.uint8)
    L = rng.integers(0, 256, (nl, 32), dtype=np.uint8)
    k = min(nl, nr) // 2
    if k:
        L[:k] = sm.flip_bits(rng, R[rng.integers(0, nr, k)], 0.05)
    if nr > 3:
        R[nr // 2] = R[1]   # exact duplicate: tie order of knnMatch
    g1, t1, d1 = stereo_knn_ratio(L, R)
    g2, t2, d2 = om.stereo_knn_ratio(L, R)
    assert g1 == g2
    np.testing.assert_array_equal(t1, t2)
    np.testing.assert_array_equal(d1, d2)


def test_empty_inputs(gpu, om):
    rng = np.random.default_rng(0)
    F = sm.synth_frame(rng, 0)
    m = ORBmatcher()
    mvp = np.zeros(0, np.int32)
    assert m.SearchByProjectionLocalMap(F, mvp, mvp, sm.synth_local_map(rng, F, 10)) == 0
    F = sm.synth_frame(rng, 50)
    mvp = np.full(50, -1, np.int32)
    assert m.SearchByProjectionLocalMap(F, mvp, np.zeros(50, np.int32), np.zeros(0, sm.MAP_POINT_DTYPE)) == 0
    assert (mvp == -1).all()
    g, t, d = stereo_knn_ratio(np.zeros((0, 32), np.uint8), np.zeros((5, 32), np.uint8))
    assert g == 0 and len(t) == 0


class _GpuAsOracle:
    """The product ORBmatcher behind the oracle-style call names used by the fixture runner."""

    def __init__(self, nnratio, checkOri):
        self.m = ORBmatcher(nnratio, checkOri)

    def sbp_local(self, F, mvp, obs, mps, th, bFar=False, thFar=50.0):
        return self.m.SearchByProjectionLocalMap(F, mvp, obs, mps, th, bFar, thFar)

    def sbp_lastframe(self, F, mvp, obs, pts, th, fw, bw):
        return self.m.SearchByProjectionLastFrame(F, mvp, obs, pts, th, fw, bw)

    def sbp_kf(self, F, mvp, pts, th, orbdist):
        return self.m.SearchByProjectionKeyFrame(F, mvp, pts, th, orbdist)

    def search_for_init(self, F1, F2, prev, m12, window):
        return self.m.SearchForInitialization(F1, F2, prev, m12, window)

    def search_by_bow(self, kk, kd, kmp, fk, F, ff):
        return self.m.SearchByBoW(kk, kd, kmp, fk, F, ff)


def test_gpu_matcher_golden(gpu):
    """The HIP matchers reproduce the committed per-query fixtures (tests/golden/matcher_golden.npz)."""
    import importlib.util
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    spec = importlib.util.spec_from_file_location("make_matcher_golden",
                                                  os.path.join(here, "golden", "make_matcher_golden.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    gold = np.load(os.path.join(here, "golden", "matcher_golden.npz"), allow_pickle=False)
    for name, kind, d in mod.cases():
        assert np.array_equal(mod.input_digest(kind, d), gold[name + "_in"]), f"{name}: generator drifted"
        if kind == "knn":
            res = stereo_knn_ratio(d["L"], d["R"])
        else:
            res = mod.run(_GpuAsOracle, kind, d)
        assert res[0] == int(gold[name + "_n"][0]), name
        for i, a in enumerate(res[1:]):
            assert np.array_equal(np.asarray(a), gold[f"{name}_out{i}"]), f"{name} output {i}"


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_is_in_frustum(gpu, om, seed):
    """Frame::isInFrustum + PredictScale on the device: every tracking field bit-exact."""
    from orb_slam3_ros_amd.matcher import is_in_frustum
    rng = np.random.default_rng(seed)
    F = sm.synth_frame(rng, 1000)
    cam = sm.synth_camera(rng)
    pts = sm.synth_local_map_3d(rng, F, cam, 50_000)
    ng, tg = is_in_frustum(F, cam, pts)
    no, to = om.is_in_frustum(F, cam, pts)
    assert ng == no and no > 1000
    inv = (to["flags"] & sm.MP_IN_VIEW) != 0
    np.testing.assert_array_equal(tg["flags"], to["flags"])
    for f in ("proj_x", "proj_y", "proj_xr", "depth", "view_cos"):
        np.testing.assert_array_equal(tg[f][inv].view(np.uint32), to[f][inv].view(np.uint32), err_msg=f)
    np.testing.assert_array_equal(tg["scale_level"][inv], to["scale_level"][inv])
    np.testing.assert_array_equal(tg["desc"], to["desc"])


@pytest.mark.parametrize("th", [1, 3, 15])
@pytest.mark.parametrize("seed", [4, 5])
def test_search_local_points(gpu, om, th, seed):
    """Tracking::SearchLocalPoints' projection + SearchByProjection fused on the device."""
    from orb_slam3_ros_amd.matcher import search_local_points
    rng = np.random.default_rng(seed)
    F = sm.synth_frame(rng, 1000)
    cam = sm.synth_camera(rng)
    pts = sm.synth_local_map_3d(rng, F, cam, 100_000)
    mvp0, obs = sm.initial_slots(rng, F.N)
    a, b = mvp0.copy(), mvp0.copy()
    ng, tg = search_local_points(F, cam, pts, a, obs, th)
    no, to = om.search_local_points(F, cam, pts, b, obs, th)
    assert (ng, tg) == (no, to) and no > 0
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("npts,th", [(1500, 1), (100_000, 1), (100_000, 15), (0, 1)],
                         ids=["block", "multi", "band", "empty"])
def test_search_local_points_track(gpu, om, npts, th):
    """orbfe_search_local_points_track (the shim's SearchLocalPoints): the same slots and counts as
    the fused search, plus every point's isInFrustum record bit-exact against the oracle's
    projection, whichever search kernel ran (one workgroup, multi-block lists, bands); a frame with no
    keypoints still projects every point (the reference's loop runs regardless)."""
    from orb_slam3_ros_amd.matcher import search_local_points
    rng = np.random.default_rng(90 + npts % 7 + th)
    F = sm.synth_frame(rng, 1000)
    cam = sm.synth_camera(rng)
    pts = sm.synth_local_map_3d(rng, F, cam, max(npts, 800))[:npts] if npts else sm.synth_local_map_3d(rng, F, cam, 800)
    mvp0, obs = sm.initial_slots(rng, F.N)
    if npts == 0:   # no keypoints in the frame, 800 points
        F = sm.synth_frame(rng, 0)
        mvp0, obs = np.zeros(0, np.int32), np.zeros(0, np.int32)
    a, b = mvp0.copy(), mvp0.copy()
    ng, tg, rec = search_local_points(F, cam, pts, a, obs, th, track=True)
    no, to = om.search_local_points(F, cam, pts, b, obs, th)
    assert (ng, tg) == (no, to)
    np.testing.assert_array_equal(a, b)
    n2, ref = om.is_in_frustum(F, cam, pts)
    assert n2 == tg and len(rec) == len(pts)
    inv = (ref["flags"] & sm.MP_IN_VIEW) != 0
    np.testing.assert_array_equal(rec["flags"], ref["flags"])
    for f in ("proj_x", "proj_y", "proj_xr", "depth", "view_cos"):
        np.testing.assert_array_equal(rec[f][inv].view(np.uint32), ref[f][inv].view(np.uint32), err_msg=f)
    np.testing.assert_array_equal(rec["scale_level"][inv], ref["scale_level"][inv])


@pytest.mark.parametrize("th", [1, 3, 15])
def test_sbp_local_device_resident(gpu, om, th):
    """orbfe_search_by_projection_local_device (records, slots and frame in HBM) == the oracle."""
    import torch
    from orb_slam3_ros_amd.matcher import DeviceMatchFrame, search_by_projection_local_device
    F, mps, mvp0, obs = _local_case(777, 1000, 50_000)
    Fd = DeviceMatchFrame(F, gpu)
    mvp_t = torch.from_numpy(mvp0.copy()).to(gpu)
    obs_t = torch.from_numpy(obs.copy()).to(gpu)
    mps_t = torch.from_numpy(mps.view(np.uint8).reshape(-1).copy()).to(gpu)
    ng = search_by_projection_local_device(Fd, mvp_t, obs_t, mps_t, th)
    mvp_o = mvp0.copy()
    no = om.OracleMatcher(0.8).sbp_local(F, mvp_o, obs, mps, th)
    assert ng == no and no > 0
    np.testing.assert_array_equal(mvp_t.cpu().numpy(), mvp_o)


def test_search_local_points_device_resident(gpu, om):
    import torch
    from orb_slam3_ros_amd.matcher import DeviceMatchFrame, search_local_points_device
    rng = np.random.default_rng(31)
    F = sm.synth_frame(rng, 1000)
    cam = sm.synth_camera(rng)
    pts = sm.synth_local_map_3d(rng, F, cam, 20000)
    mvp0, obs = sm.initial_slots(rng, F.N, 0.1)
    Fd = DeviceMatchFrame(F, gpu)
    mvp_t = torch.from_numpy(mvp0.copy()).to(gpu)
    obs_t = torch.from_numpy(obs.copy()).to(gpu)
    pts_t = torch.from_numpy(pts.view(np.uint8).reshape(-1).copy()).to(gpu)
    ng, ntm_g = search_local_points_device(Fd, cam, pts_t, mvp_t, obs_t, 1.0)
    mvp_o = mvp0.copy()
    no, ntm_o = om.search_local_points(F, cam, pts, mvp_o, obs, 1.0)
    assert (ng, ntm_g) == (no, ntm_o) and no > 0
    np.testing.assert_array_equal(mvp_t.cpu().numpy(), mvp_o)


# ---- two-camera frames (Frame.Nleft != -1, KannalaBrandt8 stereo: config 4's tracking path) ----
def _two_case(seed, nl=1000, nr=950, n_mps=20000, slots=0.15):
    rng = np.random.default_rng(seed)
    F = sm.synth_frame_two(rng, nl, nr)
    mps = sm.synth_local_map_two(rng, F, n_mps)
    mvp, obs = sm.initial_slots(rng, F.N, slots)
    return rng, F, mps, mvp, obs


@pytest.mark.parametrize("seed", [61, 62])
@pytest.mark.parametrize("th", [1, 3, 15])
def test_sbp_local_two_cams(gpu, om, seed, th):
    """SearchByProjection(F, vpMapPoints) with Nleft != -1 (ORBmatcher.cc:62-209): left search,
    mvLeftToRightMatch partner, right-grid search, mvRightToLeftMatch partner."""
    _, F, mps, mvp0, obs = _two_case(seed)
    for ratio, bfar in ((0.8, False), (0.6, True)):
        a, b = mvp0.copy(), mvp0.copy()
        ng = ORBmatcher(ratio).SearchByProjectionLocalMap(F, a, obs, mps, th, bfar, 20.0)
        no = om.OracleMatcher(ratio).sbp_local(F, b, obs, mps, th, bfar, 20.0)
        assert ng == no and no > 0
        np.testing.assert_array_equal(a, b)


def test_sbp_local_two_cams_dense(gpu, om):
    """Few keypoints, many competing points with Observations() == 0 and dense stereo links: long
    ordered chains through both cameras' slots."""
    rng = np.random.default_rng(65)
    F = sm.synth_frame_two(rng, 150, 140, w=120, h=90, stereo_frac=0.9)
    mps = sm.synth_local_map_two(rng, F, 8000, copy_frac=0.9, flip_p=0.02)
    mps["observations"] = np.where(rng.random(len(mps)) < 0.5, 0, mps["observations"])
    mvp0, obs = np.full(F.N, -1, np.int32), np.zeros(F.N, np.int32)
    for th in (1, 3):
        a, b = mvp0.copy(), mvp0.copy()
        ng = ORBmatcher(0.8).SearchByProjectionLocalMap(F, a, obs, mps, th)
        no = om.OracleMatcher(0.8).sbp_local(F, b, obs, mps, th)
        assert ng == no
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("nl,nr,n_mps,th", [
    (1000, 950, 1500, 1),     # the one-workgroup path (k_sbp_block4): <= 2048 keypoints and points
    (1000, 950, 2000, 3),
    (1000, 950, 1200, 15),
    (1024, 1024, 2048, 3),    # its limits
    (1000, 950, 2049, 3),     # one point past them: the multi-launch passes
])
def test_sbp_local_two_cams_block(gpu, om, nl, nr, n_mps, th):
    """SearchByProjection(F, vpMapPoints) with Nleft != -1 (ORBmatcher.cc:62-209) through the
    one-workgroup search and across its size limits, against the oracle: ratio 0.8 / 0.6, bFarPoints."""
    _, F, mps, mvp0, obs = _two_case(nl + nr + n_mps + th, nl, nr, n_mps)
    for ratio, bfar in ((0.8, False), (0.6, True)):
        a, b = mvp0.copy(), mvp0.copy()
        ng = ORBmatcher(ratio).SearchByProjectionLocalMap(F, a, obs, mps, th, bfar, 20.0)
        no = om.OracleMatcher(ratio).sbp_local(F, b, obs, mps, th, bfar, 20.0)
        assert ng == no and no > 0
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("n_mps", [600, 2000])
def test_sbp_local_two_cams_block_dense(gpu, om, n_mps):
    """k_sbp_block4 under competition: few keypoints, dense stereo links, half the points with
    Observations() == 0 (their slots stay open to later points, partner writes replace holders); at
    2000 points a slot can collect more writers in a pass than the block tracks, which must hand the
    search to the multi-launch form with nothing written."""
    rng = np.random.default_rng(67 + n_mps)
    F = sm.synth_frame_two(rng, 150, 140, w=120, h=90, stereo_frac=0.9)
    mps = sm.synth_local_map_two(rng, F, n_mps, copy_frac=0.9, flip_p=0.02)
    mps["observations"] = np.where(rng.random(len(mps)) < 0.5, 0, mps["observations"])
    mvp0, obs = sm.initial_slots(rng, F.N, 0.2)
    for th in (1, 3):
        a, b = mvp0.copy(), mvp0.copy()
        ng = ORBmatcher(0.8).SearchByProjectionLocalMap(F, a, obs, mps, th)
        no = om.OracleMatcher(0.8).sbp_local(F, b, obs, mps, th)
        assert ng == no
        np.testing.assert_array_equal(a, b)


def test_search_local_points_rig_block(gpu, om):
    """Tracking::SearchLocalPoints on a two-camera fisheye frame with a Tracking-sized local map
    (<= 2048 points): the device projection, then k_sbp_block4."""
    from orb_slam3_ros_amd.matcher import search_local_points
    rng, F, cam, rig, pts = _rig_case(93, True, 1800)
    mvp0, obs = sm.initial_slots(rng, F.N, 0.15)
    for th, ratio, bfar in ((1, 0.8, False), (3, 0.6, True)):
        a, b = mvp0.copy(), mvp0.copy()
        ng = search_local_points(F, cam, pts, a, obs, th, bfar, 10.0, ratio, rig=rig)
        no = om.search_local_points(F, cam, pts, b, obs, th, bfar, 10.0, ratio, rig=rig)
        assert ng == no and no[0] > 0
        np.testing.assert_array_equal(a, b)
    # the device-resident form (frame, slots and points in HBM)
    import torch
    from orb_slam3_ros_amd.matcher import DeviceMatchFrame, search_local_points_device
    Fd = DeviceMatchFrame(F, gpu)
    mvp_t = torch.from_numpy(mvp0.copy()).to(gpu)
    obs_t = torch.from_numpy(obs.copy()).to(gpu)
    pts_t = torch.from_numpy(pts.view(np.uint8).reshape(-1).copy()).to(gpu)
    ng, ntm_g = search_local_points_device(Fd, cam, pts_t, mvp_t, obs_t, 3.0, rig=rig)
    mvp_o = mvp0.copy()
    no, ntm_o = om.search_local_points(F, cam, pts, mvp_o, obs, 3.0, rig=rig)
    assert (ng, ntm_g) == (no, ntm_o) and no > 0
    np.testing.assert_array_equal(mvp_t.cpu().numpy(), mvp_o)


def test_sbp_local_two_cams_device_resident(gpu, om):
    import torch
    from orb_slam3_ros_amd.matcher import DeviceMatchFrame, search_by_projection_local_device
    _, F, mps, mvp0, obs = _two_case(66)
    Fd = DeviceMatchFrame(F, gpu)
    mvp_t = torch.from_numpy(mvp0.copy()).to(gpu)
    obs_t = torch.from_numpy(obs.copy()).to(gpu)
    mps_t = torch.from_numpy(mps.view(np.uint8).reshape(-1).copy()).to(gpu)
    ng = search_by_projection_local_device(Fd, mvp_t, obs_t, mps_t, 3.0)
    mvp_o = mvp0.copy()
    no = om.OracleMatcher(0.8).sbp_local(F, mvp_o, obs, mps, 3.0)
    assert ng == no and no > 0
    np.testing.assert_array_equal(mvp_t.cpu().numpy(), mvp_o)


@pytest.mark.parametrize("seed", [71, 72, 73])
@pytest.mark.parametrize("mode", ["none", "forward", "backward"])
@pytest.mark.parametrize("check_ori", [True, False])
def test_sbp_lastframe_two_cams(gpu, om, seed, mode, check_ori):
    """SearchByProjection(CurrentFrame, LastFrame) with CurrentFrame.Nleft != -1 (:1727-1858)."""
    rng = np.random.default_rng(seed)
    F = sm.synth_frame_two(rng, 1200, 1100)
    pts, ruv = sm.synth_proj_points_two(rng, F, 1500)
    mvp0, obs = sm.initial_slots(rng, F.N, 0.2)
    fw, bw = mode == "forward", mode == "backward"
    for th in (7, 15):
        a, b = mvp0.copy(), mvp0.copy()
        ng = ORBmatcher(0.9, check_ori).SearchByProjectionLastFrameStereo(F, a, obs, pts, ruv, th, fw, bw)
        no = om.OracleMatcher(0.9, check_ori).sbp_lastframe_stereo(F, b, obs, pts, ruv, th, fw, bw)
        assert ng == no and no > 0
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("nl,nr,npts,copy_frac", [
    (1000, 900, 1500, 0.8),    # the one-workgroup path (k_sbp_block2): n <= 2048, <= 2048 points
    (1024, 1024, 2048, 0.8),   # its limits
    (300, 280, 2000, 0.97),    # ~7 points per keypoint: entry lists (4 keys) run out, re-enumeration
    (1100, 1000, 2049, 0.8),   # one point past the block form: the multi-launch passes
    (1030, 1019, 1200, 0.8),   # one keypoint past it
])
def test_sbp_lastframe_two_cams_block(gpu, om, nl, nr, npts, copy_frac):
    """SearchByProjection(CurrentFrame, LastFrame) for a two-camera frame through the one-workgroup
    search (k_sbp_block2) and across its size limits, against the oracle's literal loop
    (ORBmatcher.cc:1695-1884): th 7 / 15, checkOri on and off, all three level filters."""
    rng = np.random.default_rng(nl + nr + npts)
    F = sm.synth_frame_two(rng, nl, nr)
    pts, ruv = sm.synth_proj_points_two(rng, F, npts, copy_frac=copy_frac)
    mvp0, obs = sm.initial_slots(rng, F.N, 0.2)
    for th, check_ori, fw, bw in [(7, True, False, False), (15, False, True, False), (7, True, False, True)]:
        a, b = mvp0.copy(), mvp0.copy()
        ng = ORBmatcher(0.9, check_ori).SearchByProjectionLastFrameStereo(F, a, obs, pts, ruv, th, fw, bw)
        no = om.OracleMatcher(0.9, check_ori).sbp_lastframe_stereo(F, b, obs, pts, ruv, th, fw, bw)
        assert ng == no and no > 0, (th, ng, no)
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("kind,nl,nr,npts", [
    ("pinhole", 1000, 0, 1500),   # k_sbp_block<1> on device-projected records
    ("pinhole", 1000, 0, 2100),   # beyond the block form: projected, then the multi-launch passes
    ("kb8", 1000, 950, 1500),     # two cameras: k_sbp_block2 with both cameras' projections on the device
    ("kb8", 1000, 950, 2100),
])
def test_sbp_lastframe_pose(gpu, om, kind, nl, nr, npts):
    """SearchByProjection(CurrentFrame, LastFrame) with the projection on the device
    (orbfe_search_by_projection_lastframe_pose, ORBmatcher.cc:1695-1718, 1794-1796: Sophus Tcw * x3Dw,
    invzc in double, mpCamera->project for both cameras) against the oracle's projection + loop."""
    from orb_slam3_ros_amd.matcher import CameraModel, Pose
    rng = np.random.default_rng(nl + nr + npts + (7 if kind == "kb8" else 0))
    if kind == "kb8":
        F = sm.synth_frame_two(rng, nl, nr)
        model = CameraModel.make("kb8", *sm.TUMVI_LEFT[:4], sm.TUMVI_LEFT[4])
        Trl = Pose.se3(*sm.synth_pose(rng, 1.0, 0.05))
    else:
        F = sm.synth_frame(rng, nl)
        model = CameraModel.make("pinhole", 458.654, 457.296, 367.215, 248.375)
        Trl = None
    R, t = sm.synth_pose(rng)
    Tcw = Pose.se3(R, t)
    pts = sm.synth_last_points(rng, F, model, R, t, npts)
    mvp0, obs = sm.initial_slots(rng, F.N, 0.2)
    total = 0
    for th, check_ori, fw, bw in [(7, True, False, False), (15, False, True, False), (7, True, False, True)]:
        a, b = mvp0.copy(), mvp0.copy()
        ng = ORBmatcher(0.9, check_ori).SearchByProjectionLastFramePose(F, a, obs, pts, Tcw, model, th, fw, bw, Trl)
        no = om.OracleMatcher(0.9, check_ori).sbp_lastframe_pose(F, b, obs, pts, Tcw, model, th, fw, bw, Trl)
        assert ng == no, (th, ng, no)
        np.testing.assert_array_equal(a, b)
        total += no
    assert total > 100


def test_sbp_two_cams_keyframe_left_grid(gpu, om):
    """SearchByProjection(CurrentFrame, pKF) has no right-camera branch: a two-camera frame is
    searched through its left grid only (GetFeaturesInArea's default bRight = false)."""
    rng = np.random.default_rng(74)
    F = sm.synth_frame_two(rng, 900, 900)
    left = sm.MatchFrame(F.keys[:900], F.desc[:900], F.bounds, F.scale_factors)
    pts = sm.synth_proj_points(rng, left, 1000, copy_frac=0.7)
    mvp0, _ = sm.initial_slots(rng, F.N, 0.2)
    a, b = mvp0.copy(), mvp0.copy()
    ng = ORBmatcher(0.9, True).SearchByProjectionKeyFrame(F, a, pts, 10, 100)
    # oracle: the same search over the left rows (the right rows are never candidates)
    bl = b[:900].copy()
    no = om.OracleMatcher(0.9, True).sbp_kf(left, bl, pts, 10, 100)
    b[:900] = bl
    assert ng == no and no > 0
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("seed", [81, 82, 83])
@pytest.mark.parametrize("check_ori", [True, False])
def test_search_by_bow_two_cams(gpu, om, seed, check_ori):
    """SearchByBoW(pKF, F) with F.Nleft != -1 (:288-386, the right match's "|| true")."""
    rng = np.random.default_rng(seed)
    KF = sm.synth_frame(rng, 1000, 512, 512, stereo=False)
    F = sm.synth_frame_two(rng, 900, 900)
    # F's features: noisy copies of KF features on both cameras
    src = np.where(rng.random(F.N) < 0.7, rng.integers(0, KF.N, F.N), -1)
    cp = src >= 0
    F.desc[cp] = sm.flip_bits(rng, KF.desc[src[cp]], 0.05)
    F.keys["angle"][cp] = np.mod(KF.keys["angle"][src[cp]] + 20 + rng.normal(0, 3, int(cp.sum())), 360)
    kf_mp = np.where(rng.random(KF.N) < 0.25, -1, np.arange(KF.N) + 100).astype(np.int32)
    for words in (50, 400):
        fk, ff = sm.synth_bow(rng, words, KF, F, src)
        ng, out_g = ORBmatcher(0.75, check_ori).SearchByBoW(KF.keys, KF.desc, kf_mp, fk, F, ff)
        no, out_o = om.OracleMatcher(0.75, check_ori).search_by_bow(KF.keys, KF.desc, kf_mp, fk, F, ff)
        assert ng == no and no > 0
        np.testing.assert_array_equal(out_g, out_o)
        assert (out_o[900:] >= 0).any()   # right-camera matches happened


def test_two_cams_input_rules(gpu):
    """Two-camera frames need their right-view inputs: the last-frame search refuses one without the
    right projections, SearchForInitialization (monocular initialisation, Nleft == -1 only) refuses it."""
    from orb_slam3_ros_amd._lib import OrbfeError
    rng = np.random.default_rng(90)
    F = sm.synth_frame_two(rng, 50, 40)
    pts = sm.synth_proj_points(rng, sm.MatchFrame(F.keys[:50], F.desc[:50], F.bounds, F.scale_factors), 20)
    mvp, obs = np.full(F.N, -1, np.int32), np.zeros(F.N, np.int32)
    with pytest.raises(OrbfeError):   # last-frame search without the right projections
        ORBmatcher(0.9).SearchByProjectionLastFrame(F, mvp, obs, pts, 7, False, False)
    with pytest.raises(OrbfeError):
        ORBmatcher(0.9).SearchForInitialization(F, F, np.zeros((F.N, 2), np.float32), np.zeros(F.N, np.int32))


# ---- Frame::isInFrustum with KannalaBrandt8 cameras (SURVEY §8f.1 for config 4's TUM-VI rig) ----
def _rig_case(seed, two, n_pts, nl=1000, nr=950):
    rng = np.random.default_rng(seed)
    F = sm.synth_frame_two(rng, nl, nr) if two else sm.synth_frame(rng, nl, 512, 512, stereo=False)
    cam = sm.synth_camera(rng, rot_deg=20.0)
    rig = sm.synth_rig(cam, two)
    pts = sm.synth_local_map_3d_rig(rng, F, cam, n_pts, two=two)
    return rng, F, cam, rig, pts


@pytest.mark.parametrize("two", [False, True], ids=["mono_kb8", "two_cams"])
@pytest.mark.parametrize("seed", [1, 2])
def test_is_in_frustum_rig(gpu, om, seed, two):
    """isInFrustum (Nleft == -1 with a KannalaBrandt8 mpCamera, or isInFrustumChecks left + right,
    Frame.cc:512-586, 1168-1242) on the device: flags and every field of each passing view bit-exact."""
    from orb_slam3_ros_amd.matcher import is_in_frustum
    _, F, cam, rig, pts = _rig_case(seed, two, 50_000)
    ng, tg = is_in_frustum(F, cam, pts, rig)
    no, to = om.is_in_frustum(F, cam, pts, rig)
    assert ng == no and no > 1000
    np.testing.assert_array_equal(tg["flags"], to["flags"])
    inv = (to["flags"] & sm.MP_IN_VIEW) != 0
    for f in ("proj_x", "proj_y", "depth", "view_cos") + (() if two else ("proj_xr",)):
        np.testing.assert_array_equal(tg[f][inv].view(np.uint32), to[f][inv].view(np.uint32), err_msg=f)
    np.testing.assert_array_equal(tg["scale_level"], to["scale_level"])
    # mTrackDepth is written only by a passing left view; every other point keeps its previous value
    # (orbfe_map_point_3d.track_depth), which bFarPoints reads for right-only points
    np.testing.assert_array_equal(tg["depth"].view(np.uint32), to["depth"].view(np.uint32))
    if two:
        assert (~inv & ((to["flags"] & sm.MP_IN_VIEW_R) != 0) & (to["depth"] > 10.0)).sum() > 100
        invr = (to["flags"] & sm.MP_IN_VIEW_R) != 0
        assert invr.sum() > 1000
        for f in ("proj_xr", "proj_yr", "view_cos_r"):
            np.testing.assert_array_equal(tg[f][invr].view(np.uint32), to[f][invr].view(np.uint32), err_msg=f)
        np.testing.assert_array_equal(tg["scale_level_r"], to["scale_level_r"])


@pytest.mark.parametrize("two", [False, True], ids=["mono_kb8", "two_cams"])
@pytest.mark.parametrize("th", [1, 3, 15])
def test_search_local_points_rig(gpu, om, th, two):
    """Tracking::SearchLocalPoints (Tracking.cc:3407-3452) on a fisheye frame: device projection +
    SearchByProjection's Nleft branches (ORBmatcher.cc:43-213) == the oracle, ratio 0.8 and 0.6 with
    bFarPoints."""
    from orb_slam3_ros_amd.matcher import search_local_points
    rng, F, cam, rig, pts = _rig_case(70 + th, two, 60_000)
    mvp0, obs = sm.initial_slots(rng, F.N, 0.15)
    for ratio, bfar in ((0.8, False), (0.6, True)):
        a, b = mvp0.copy(), mvp0.copy()
        ng = search_local_points(F, cam, pts, a, obs, th, bfar, 10.0, ratio, rig=rig)
        no = om.search_local_points(F, cam, pts, b, obs, th, bfar, 10.0, ratio, rig=rig)
        assert ng == no and no[0] > 0 and no[1] > 1000
        np.testing.assert_array_equal(a, b)


def test_search_local_points_rig_device_resident(gpu, om):
    import torch
    from orb_slam3_ros_amd.matcher import DeviceMatchFrame, search_local_points_device
    rng, F, cam, rig, pts = _rig_case(91, True, 40_000)
    mvp0, obs = sm.initial_slots(rng, F.N, 0.1)
    Fd = DeviceMatchFrame(F, gpu)
    mvp_t = torch.from_numpy(mvp0.copy()).to(gpu)
    obs_t = torch.from_numpy(obs.copy()).to(gpu)
    pts_t = torch.from_numpy(pts.view(np.uint8).reshape(-1).copy()).to(gpu)
    ng, ntm_g = search_local_points_device(Fd, cam, pts_t, mvp_t, obs_t, 3.0, rig=rig)
    mvp_o = mvp0.copy()
    no, ntm_o = om.search_local_points(F, cam, pts, mvp_o, obs, 3.0, rig=rig)
    assert (ng, ntm_g) == (no, ntm_o) and no > 0
    np.testing.assert_array_equal(mvp_t.cpu().numpy(), mvp_o)


def test_two_cams_frustum_needs_rig(gpu):
    """A two-camera frame through the pinhole-only entry points is refused (no right camera)."""
    from orb_slam3_ros_amd import _lib
    from orb_slam3_ros_amd.matcher import is_in_frustum, search_local_points
    rng, F, cam, rig, pts = _rig_case(5, True, 100)
    mvp, obs = sm.initial_slots(rng, F.N, 0.1)
    with pytest.raises(_lib.OrbfeError):
        is_in_frustum(F, cam, pts)
    with pytest.raises(_lib.OrbfeError):
        search_local_points(F, cam, pts, mvp, obs, 1.0)


@pytest.mark.parametrize("n_kp", [2048, 2049])
@pytest.mark.parametrize("th", [1, 5])
def test_sbp_local_band_edges(gpu, om, n_kp, th):
    """k_sbp_band's (octave, 8-row band) candidate runs against the reference's GetFeaturesInArea:
    keypoints and projections on integer and band-boundary rows (y = 8k, y +- R exactly on a band
    edge), keypoints outside the grid's bounds (PosInGrid false: never candidates), tied distances
    (duplicated descriptors: the enumeration order decides), at the band kernel's size limit (2048
    keypoints) and one past it (the grid-walk kernels)."""
    rng = np.random.default_rng(4242 + n_kp + th)
    F0 = sm.synth_frame(rng, n_kp)
    k = F0.keys.copy()
    k["y"][: n_kp // 3] = (8.0 * rng.integers(0, 60, n_kp // 3)).astype(np.float32)     # on band edges
    k["x"][: n_kp // 4] = np.round(k["x"][: n_kp // 4]).astype(np.float32)
    k["x"][-20:] = np.float32(751.5)   # round((x - minx) * 64 / 747) = 64: outside the grid
    desc = F0.desc.copy()
    desc[1::7] = desc[0::7][: len(desc[1::7])]   # exact duplicates: distance ties
    F = MatchFrame(k, desc, (0.0, 747.0, 0.0, 480.0), F0.scale_factors, F0.uright, F0.mbf)
    mps = sm.synth_local_map(rng, F, 30000, copy_frac=0.5)
    # projections exactly on band rows, and y +- R on a band edge for level-0 radius 2.5 * th
    sel = rng.random(len(mps)) < 0.3
    mps["proj_y"][sel] = (8.0 * rng.integers(0, 60, int(sel.sum()))).astype(np.float32)
    sel2 = rng.random(len(mps)) < 0.1
    mps["proj_y"][sel2] = (8.0 * rng.integers(1, 59, int(sel2.sum())) + 2.5 * th).astype(np.float32)
    mps["view_cos"][sel2] = 0.9995
    mps["scale_level"][sel2] = 0
    mvp0, obs = sm.initial_slots(rng, F.N, 0.1)
    a, b = mvp0.copy(), mvp0.copy()
    ng = ORBmatcher(0.8).SearchByProjectionLocalMap(F, a, obs, mps, th)
    no = om.OracleMatcher(0.8).sbp_local(F, b, obs, mps, th)
    assert ng == no and no > 0
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("nq", [2048, 2049])
def test_sbp_block_limit(gpu, om, nq):
    """The single-workgroup fixed point (k_sbp_block, up to 2048 queries) and the multi-block passes
    one query past it, for the three SearchByProjection variants on one dense case (duplicated
    descriptors and map points: long "later points see earlier assignments" chains)."""
    rng = np.random.default_rng(900 + nq)
    F = sm.synth_frame(rng, 1800)
    F.desc[1::5] = F.desc[0::5][: len(F.desc[1::5])]
    mps = sm.synth_local_map(rng, F, nq, copy_frac=0.8, flip_p=0.02)
    pts = sm.synth_proj_points(rng, F, nq, copy_frac=0.8)
    mvp0, obs = sm.initial_slots(rng, F.N, 0.15)
    for th in (1, 5):
        a, b = mvp0.copy(), mvp0.copy()
        assert ORBmatcher(0.8).SearchByProjectionLocalMap(F, a, obs, mps, th) == \
            om.OracleMatcher(0.8).sbp_local(F, b, obs, mps, th)
        np.testing.assert_array_equal(a, b)
    for mode in ("none", "forward", "backward"):
        a, b = mvp0.copy(), mvp0.copy()
        fw, bw = mode == "forward", mode == "backward"
        assert ORBmatcher(0.9, True).SearchByProjectionLastFrame(F, a, obs, pts, 7, fw, bw) == \
            om.OracleMatcher(0.9, True).sbp_lastframe(F, b, obs, pts, 7, fw, bw)
        np.testing.assert_array_equal(a, b)
    a, b = mvp0.copy(), mvp0.copy()
    assert ORBmatcher(0.9, True).SearchByProjectionKeyFrame(F, a, pts, 10, 100) == \
        om.OracleMatcher(0.9, True).sbp_kf(F, b, pts, 10, 100)
    np.testing.assert_array_equal(a, b)


def _crowded_case(seed, n_kp=1200, n_mps=6000, per=12):
    """Clusters of `per` keypoints within a few pixels whose descriptors form a ladder (keypoint i
    differs from keypoint 0 in 6 i bits) on alternating octaves 0 / 1, and per cluster `per` + 4
    map points (level 1, Observations() > 0) with keypoint 0's descriptor: the j-th of them takes
    keypoint j (alternating octaves skip the ratio test), so from the 9th on every point's 8-key
    candidate list is taken by earlier points and k_sbp_multi re-enumerates its window."""
    rng = np.random.default_rng(seed)
    F = sm.synth_frame(rng, n_kp)
    k = F.keys.copy()
    desc = F.desc.copy()
    ncl = n_kp // per
    cx = rng.uniform(40, 700, ncl).astype(np.float32)
    cy = rng.uniform(40, 440, ncl).astype(np.float32)
    for c in range(ncl):
        sl = slice(c * per, (c + 1) * per)
        k["x"][sl] = cx[c] + rng.uniform(-2.0, 2.0, per).astype(np.float32)
        k["y"][sl] = cy[c] + rng.uniform(-2.0, 2.0, per).astype(np.float32)
        k["octave"][sl] = np.arange(per) % 2
        bits = np.unpackbits(desc[c * per])
        order = rng.permutation(256)
        for i in range(per):
            b = bits.copy()
            b[order[:6 * i]] ^= 1
            desc[c * per + i] = np.packbits(b)
    F = MatchFrame(k, desc, F.bounds, F.scale_factors, None, F.mbf)
    mps = sm.synth_local_map(rng, F, n_mps, copy_frac=0.0)
    m = min(n_mps, ncl * (per + 4))
    cl = np.arange(m) // (per + 4)
    mps["proj_x"][:m] = cx[cl]
    mps["proj_y"][:m] = cy[cl]
    mps["scale_level"][:m] = 1
    mps["view_cos"][:m] = 0.995            # radius 4 * th * scale[1]
    mps["flags"][:m] = sm.MP_IN_VIEW
    mps["observations"][:m] = rng.integers(1, 9, m)
    mps["desc"][:m] = desc[cl * per]
    perm = rng.permutation(n_mps)           # interleave the crowded points with the rest
    return F, mps[perm]


@pytest.mark.parametrize("th", [1, 3])
def test_sbp_multi_lists_run_out(gpu, om, th):
    """k_sbp_multi0 / k_sbp_multi (more than 2048 points, th < 4) when candidate lists run out: the
    passes re-enumerate over block 0's frame copy with their gates. Host and device-resident calls
    against the oracle."""
    import torch
    from orb_slam3_ros_amd.matcher import DeviceMatchFrame, search_by_projection_local_device
    F, mps = _crowded_case(77 + th)
    rng = np.random.default_rng(5)
    mvp0, obs = sm.initial_slots(rng, F.N, 0.05)
    a, b = mvp0.copy(), mvp0.copy()
    ng = ORBmatcher(0.8).SearchByProjectionLocalMap(F, a, obs, mps, th)
    no = om.OracleMatcher(0.8).sbp_local(F, b, obs, mps, th)
    assert ng == no and no > 0
    np.testing.assert_array_equal(a, b)
    Fd = DeviceMatchFrame(F, gpu)
    mvp_t = torch.from_numpy(mvp0.copy()).to(gpu)
    nd = search_by_projection_local_device(Fd, mvp_t, torch.from_numpy(obs.copy()).to(gpu),
                                           torch.from_numpy(mps.view(np.uint8).reshape(-1).copy()).to(gpu), th)
    torch.cuda.synchronize()
    assert nd == no
    np.testing.assert_array_equal(mvp_t.cpu().numpy(), b)


def test_sbp_multi_degenerate(gpu, om):
    """The multi-block search with nothing to do: every keypoint held by a point with observations
    (all blocked), and no point in view; both converge at pass 0 and leave the slots alone."""
    rng = np.random.default_rng(31)
    F = sm.synth_frame(rng, 1000)
    mps = sm.synth_local_map(rng, F, 5000, copy_frac=0.5)
    mvp = np.arange(F.N, dtype=np.int32) + 1
    obs = np.full(F.N, 3, np.int32)
    a = mvp.copy()
    assert ORBmatcher(0.8).SearchByProjectionLocalMap(F, a, obs, mps, 1) == 0
    np.testing.assert_array_equal(a, mvp)
    mvp0, obs0 = sm.initial_slots(rng, F.N, 0.1)
    off = mps.copy()
    off["flags"] = 0
    a, b = mvp0.copy(), mvp0.copy()
    assert ORBmatcher(0.8).SearchByProjectionLocalMap(F, a, obs0, off, 1) == \
        om.OracleMatcher(0.8).sbp_local(F, b, obs0, off, 1) == 0
    np.testing.assert_array_equal(a, b)
    # and a normal search right after (the counters the degenerate calls used are reset)
    a, b = mvp0.copy(), mvp0.copy()
    assert ORBmatcher(0.8).SearchByProjectionLocalMap(F, a, obs0, mps, 1) == \
        om.OracleMatcher(0.8).sbp_local(F, b, obs0, mps, 1)
    np.testing.assert_array_equal(a, b)


def _crowd(F, rng, k, x, y, octave=0):
    """k of F's keypoints moved into one grid cell / band bucket (within a pixel of (x, y))."""
    idx = rng.choice(F.N, k, replace=False)
    F.keys["x"][idx] = x + rng.uniform(-0.4, 0.4, k)
    F.keys["y"][idx] = y + rng.uniform(-0.4, 0.4, k)
    F.keys["octave"][idx] = octave
    return MatchFrame(F.keys, F.desc, F.bounds, F.scale_factors, F.uright, F.mbf)


def test_search_for_initialization_crowded_cell(gpu, om):
    """More than 32 of F2's level-0 keypoints in one grid cell: k_mt_grid's bitonic fallback (the
    counting sort keeps at most 32 per cell in index order)."""
    rng = np.random.default_rng(77)
    F1 = sm.synth_frame(rng, 2000, stereo=False)
    F2, _ = sm.perturbed_frame(rng, F1, shift=(3.0, -2.0), jitter=1.0, rot=8.0, flip_p=0.05, drop=0.1)
    F2 = _crowd(F2, rng, 120, 300.0, 200.0)
    prev0 = np.stack([F1.keys["x"], F1.keys["y"]], 1).astype(np.float32)
    pa, pb = prev0.copy(), prev0.copy()
    ma, mb = np.zeros(F1.N, np.int32), np.zeros(F1.N, np.int32)
    ng = ORBmatcher(0.9, True).SearchForInitialization(F1, F2, pa, ma, 100)
    no = om.OracleMatcher(0.9, True).search_for_init(F1, F2, pb, mb, 100)
    assert ng == no
    np.testing.assert_array_equal(ma, mb)
    np.testing.assert_array_equal(pa, pb)


@pytest.mark.parametrize("th", [5, 15])
def test_sbp_local_band_crowded_bucket(gpu, om, th):
    """k_sbp_band over a band index with one (octave, band) bucket of 150 keypoints (the index's
    bitonic fallback) against the oracle; 5,000 points, so the multi-block band passes run."""
    rng = np.random.default_rng(91 + th)
    F = sm.synth_frame(rng, 1000)
    F = _crowd(F, rng, 150, 400.0, 243.0, octave=1)
    mps = sm.synth_local_map(rng, F, 5000)
    mvp0, obs = sm.initial_slots(rng, F.N)
    a, b = mvp0.copy(), mvp0.copy()
    ng = ORBmatcher(0.8).SearchByProjectionLocalMap(F, a, obs, mps, th)
    no = om.OracleMatcher(0.8).sbp_local(F, b, obs, mps, th)
    assert ng == no
    np.testing.assert_array_equal(a, b)
