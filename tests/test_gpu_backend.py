"""GPU parity of the back-end ORBmatcher pieces through the C-ABI against the CPU
oracle (oracle/orb_oracle_match.cpp):
 * SearchByBoW(KF, KF) (ORBmatcher.cc:765-903): full vpMatches12 + nmatches, with and without the
   rotation check, small and large vocabulary nodes, NULL/bad map points on both sides;
 * MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:329-403): chosen row per point for set
   sizes 0..2048 (LDS-staged and global-row paths), duplicate rows (first minimum wins).
Parity is "unpinned" w.r.t. the real reference (no buildable reference, no fixtures): DESIGN.md.
"""
import numpy as np
import pytest

from orb_slam3_ros_amd import synth_match as sm
from orb_slam3_ros_amd._lib import OrbfeError
from orb_slam3_ros_amd.matcher import FeatureVector, MatchFrame, ORBmatcher, compute_distinctive_descriptors

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,n,words,check_ori", [(0, 1000, 400, True), (1, 1000, 400, False),
                                                     (2, 2000, 12, True), (3, 300, 3, True)])
def test_search_by_bow_kf(gpu, oracle_lib, seed, n, words, check_ori):
    rng = np.random.default_rng(seed)
    K1, K2, mp1, mp2, fv1, fv2 = sm.synth_kf_pair(rng, n, words)
    for ratio in (0.75, 0.9):
        ng, og = ORBmatcher(ratio, check_ori).SearchByBoWKF(K1.keys, K1.desc, mp1, fv1, K2.keys, K2.desc, mp2, fv2)
        no, oo = oracle_lib.OracleMatcher(ratio, check_ori).search_by_bow_kf(K1.keys, K1.desc, mp1, fv1, K2.keys,
                                                                              K2.desc, mp2, fv2)
        assert ng == no and no > 0
        np.testing.assert_array_equal(og, oo)


def test_search_by_bow_kf_edges(gpu, oracle_lib):
    rng = np.random.default_rng(7)
    K1, K2, mp1, mp2, fv1, fv2 = sm.synth_kf_pair(rng, 200, 20)
    m = ORBmatcher(0.75, True)
    # no shared nodes / empty feature vectors / every KF1 point NULL
    n, out = m.SearchByBoWKF(K1.keys, K1.desc, mp1, FeatureVector({1: [0]}), K2.keys, K2.desc, mp2,
                             FeatureVector({2: [0]}))
    assert n == 0 and (out == -1).all()
    n, out = m.SearchByBoWKF(K1.keys, K1.desc, mp1, FeatureVector({}), K2.keys, K2.desc, mp2, fv2)
    assert n == 0 and (out == -1).all() and len(out) == K1.N
    n, out = m.SearchByBoWKF(K1.keys, K1.desc, np.full(K1.N, -1, np.int32), fv1, K2.keys, K2.desc, mp2, fv2)
    assert n == 0 and (out == -1).all()
    # a keypoint index listed in two nodes violates the FeatureVector invariant
    with pytest.raises(OrbfeError):
        m.SearchByBoWKF(K1.keys, K1.desc, mp1, FeatureVector({1: [0], 2: [0]}), K2.keys, K2.desc, mp2, fv2)


@pytest.mark.parametrize("seed", [0, 1])
def test_distinctive_descriptors(gpu, oracle_lib, seed):
    rng = np.random.default_rng(seed)
    sizes = [0, 1, 2, 3, 4, 5, 63, 64, 65, 128, 255, 256, 257, 700, 2048] + list(rng.integers(1, 40, 2000))
    sets = sm.synth_distinctive_sets(rng, sizes, flip_p=0.15 + 0.1 * seed)
    offs = np.zeros(len(sets) + 1, np.int32)
    offs[1:] = np.cumsum([len(d) for d in sets])
    desc = np.concatenate(sets)
    got = compute_distinctive_descriptors((desc, offs))
    ref = oracle_lib.distinctive_descriptors(desc, offs)
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(compute_distinctive_descriptors(sets[:20]), ref[:20])
    assert got[0] == -1


def test_distinctive_descriptors_limits(gpu):
    assert len(compute_distinctive_descriptors([])) == 0
    big = np.zeros((2049, 32), np.uint8)
    with pytest.raises(OrbfeError):
        compute_distinctive_descriptors([big])
    # all-identical rows: every median is 0, the first row wins
    np.testing.assert_array_equal(compute_distinctive_descriptors([np.ones((9, 32), np.uint8)]), [0])


# ---- SearchForTriangulation / Fuse / SearchByProjection(Sim3) / SearchBySim3 ----
@pytest.mark.parametrize("seed,coarse,only_stereo,check_ori", [(0, False, False, True), (1, True, False, True),
                                                                (2, False, False, False), (3, False, True, True)])
def test_search_for_triangulation(gpu, oracle_lib, seed, coarse, only_stereo, check_ori):
    rng = np.random.default_rng(seed)
    K1, K2, *_, c1, c2, S12, S21, src = sm.synth_sim3_pair(rng, 1500)
    if only_stereo:   # stereo keypoints on both sides (mvuRight >= 0)
        def stereo(K):
            ur = np.where(rng.random(K.N) < 0.6, K.keys["x"] - 10, -1).astype(np.float32)
            return MatchFrame(K.keys, K.desc, K.bounds, K.scale_factors, ur, K.mbf)
        K1, K2 = stereo(K1), stereo(K2)
    for words in (300, 20):
        fv1, fv2 = sm.synth_bow(rng, words, K1, K2, src)
        F12, ep = sm.fundamental_12(c1, c2)
        sg = (K2.scale_factors * K2.scale_factors).astype(np.float32)
        mp1 = np.where(rng.random(K1.N) < 0.4, 5, -1).astype(np.int32)
        mp2 = np.where(rng.random(K2.N) < 0.4, 5, -1).astype(np.int32)
        m = ORBmatcher(0.6, check_ori)
        ng, og = m.SearchForTriangulation(K1, mp1, fv1, K2, mp2, fv2, F12, ep, sg, only_stereo, coarse)
        no, oo = oracle_lib.OracleMatcher(0.6, check_ori).search_for_triangulation(K1, mp1, fv1, K2, mp2, fv2, F12,
                                                                                    ep, sg, only_stereo, coarse)
        assert ng == no
        np.testing.assert_array_equal(og, oo)
        assert no > 20


@pytest.mark.parametrize("sim3", [0, 1])
@pytest.mark.parametrize("seed,n_kp,n_pts,dup,th", [(0, 1000, 4000, 2, 3.0), (1, 2000, 20000, 3, 5.0),
                                                    (2, 500, 800, 1, 1.0)])
def test_fuse(gpu, oracle_lib, sim3, seed, n_kp, n_pts, dup, th):
    rng = np.random.default_rng(seed)
    KF, cam, pts = sm.synth_fuse_scene(rng, n_kp, n_pts, dup=dup)
    ng, big, bdg = ORBmatcher().Fuse(KF, cam, pts, th, sim3=bool(sim3))
    no, bio, bdo = oracle_lib.OracleMatcher().fuse(KF, cam, pts, th, sim3=sim3)
    assert ng == no and no > 0
    np.testing.assert_array_equal(big, bio)
    np.testing.assert_array_equal(bdg, bdo)


@pytest.mark.parametrize("with_kfs", [False, True])
@pytest.mark.parametrize("seed,dup,ratio,th", [(0, 3, 1.0, 10), (1, 2, 0.5, 10), (2, 4, 1.0, 20)])
def test_search_by_projection_sim3(gpu, oracle_lib, with_kfs, seed, dup, ratio, th):
    rng = np.random.default_rng(seed)
    KF, cam, pts = sm.synth_fuse_scene(rng, 1000, 3000, dup=dup)
    matched0 = np.full(KF.N, -1, np.int32)
    pre = rng.random(KF.N) < 0.1
    matched0[pre] = rng.choice(pts["id"], int(pre.sum()))   # spAlreadyFound: those points are skipped
    kfs = rng.integers(0, 50, len(pts)).astype(np.int32) if with_kfs else None
    mk0 = np.where(pre, 99, -1).astype(np.int32)
    mg, mkg = matched0.copy(), mk0.copy()
    ng = ORBmatcher().SearchByProjectionSim3(KF, cam, pts, mg, th, ratio, kfs, mkg if with_kfs else None)
    mo, mko = matched0.copy(), mk0.copy()
    no = oracle_lib.OracleMatcher().sbp_sim3(KF, cam, pts, mo, th, ratio, kfs, mko if with_kfs else None)
    assert ng == no and no > 0
    np.testing.assert_array_equal(mg, mo)
    if with_kfs:
        np.testing.assert_array_equal(mkg, mko)


@pytest.mark.parametrize("two", [False, True], ids=["mono_kb8", "two_cams"])
@pytest.mark.parametrize("seed,ratio,th", [(0, 1.0, 10), (1, 0.5, 20)])
def test_search_by_projection_sim3_kb8(gpu, oracle_lib, two, seed, ratio, th):
    """SearchByProjection(pKF, Scw, ...) on a KannalaBrandt8 keyframe (ORBmatcher.cc:427-523): the
    projection is pKF->mpCamera->project (:465) on the device, a two-camera keyframe is searched on
    its left grid (KeyFrame::GetFeaturesInArea(.., bRight = false)); the vpPointsKFs overload keeps
    the pinhole expression (:571-576)."""
    rng = np.random.default_rng(120 + seed + 10 * two)
    KF = sm.synth_frame_two(rng, 1000, 950) if two else sm.synth_frame(rng, 1000, 512, 512, stereo=False)
    cam = sm.synth_camera(rng, rot_deg=20.0)
    rig = sm.synth_rig(cam, two)
    pts = sm.synth_local_map_3d_rig(rng, KF, cam, 6000, two=two)
    kcam = sm.left_kf_camera(cam)
    matched0 = np.full(KF.N, -1, np.int32)
    pre = rng.random(KF.N) < 0.1
    matched0[pre] = rng.choice(pts["id"], int(pre.sum()))
    for kfs in (None, rng.integers(0, 50, len(pts)).astype(np.int32)):
        mk0 = np.where(pre, 99, -1).astype(np.int32)
        mg, mo, mkg, mko = matched0.copy(), matched0.copy(), mk0.copy(), mk0.copy()
        ng = ORBmatcher().SearchByProjectionSim3(KF, kcam, pts, mg, th, ratio, kfs, None if kfs is None else mkg,
                                                 model=rig.left)
        no = oracle_lib.OracleMatcher().sbp_sim3(KF, kcam, pts, mo, th, ratio, kfs, None if kfs is None else mko,
                                                 model=rig.left)
        assert ng == no and (no > 50 or kfs is not None)
        np.testing.assert_array_equal(mg, mo)
        np.testing.assert_array_equal(mkg, mko)
        if two:
            new = (mg >= 0) & (matched0 < 0)
            assert not new[KF.nleft:].any()   # right keypoints are never candidates
    if two:   # the pinhole entry point needs the camera model for the first overload
        with pytest.raises(OrbfeError):
            ORBmatcher().SearchByProjectionSim3(KF, kcam, pts, matched0.copy(), th, ratio)


def _as_two_cams(K, frac):
    """The keyframe's keypoints split into a left part [0, nleft) and a 'right' part (a two-camera
    keyframe, NLeft != -1, no stereo links)."""
    nl = int(K.N * frac)
    return MatchFrame(K.keys, K.desc, K.bounds, K.scale_factors, None, K.mbf, nleft=nl)


@pytest.mark.parametrize("kinds", [(True, True), (True, False), (False, True)], ids=["two_two", "two_one", "one_two"])
@pytest.mark.parametrize("seed,scale,th", [(0, 1.0, 7.5), (2, 1.3, 7.5)])
def test_search_by_sim3_two_cams(gpu, oracle_lib, kinds, seed, scale, th):
    """SearchBySim3 with keyframes that have a second camera (ORBmatcher.cc:1457-1674): every point
    (left and right keypoints) projects with the pinhole expression on pKF1's intrinsics, candidates
    come from the left grid (mvKeys) of the target keyframe."""
    rng = np.random.default_rng(300 + seed)
    K1, K2, p1, p2, c1, c2, S12, S21, src = sm.synth_sim3_pair(rng, 2000, scale=scale)
    A = _as_two_cams(K1, 0.6) if kinds[0] else K1
    B = _as_two_cams(K2, 0.7) if kinds[1] else K2
    m0 = np.full(A.N, -1, np.int32)
    pre = np.nonzero(rng.random(A.N) < 0.05)[0]
    m0[pre] = 123
    mg, mo = m0.copy(), m0.copy()
    ng = ORBmatcher().SearchBySim3(A, B, p1, p2, c1, c2, S12, S21, th, mg)
    no = oracle_lib.OracleMatcher().search_by_sim3(A, B, p1, p2, c1, c2, S12, S21, th, mo)
    assert ng == no
    np.testing.assert_array_equal(mg, mo)
    if scale == 1.0:
        assert no > 50


@pytest.mark.parametrize("seed,scale,th", [(0, 1.0, 7.5), (1, 1.0, 15.0), (2, 1.3, 7.5), (3, 0.8, 10.0)])
def test_search_by_sim3(gpu, oracle_lib, seed, scale, th):
    rng = np.random.default_rng(seed)
    K1, K2, p1, p2, c1, c2, S12, S21, src = sm.synth_sim3_pair(rng, 2000, scale=scale)
    m0 = np.full(K1.N, -1, np.int32)
    pre = np.nonzero(rng.random(K1.N) < 0.05)[0]
    m0[pre] = 123
    inv = np.full(K1.N, -1, np.int64)   # KF1 index -> the KF2 keypoint observing the same point
    inv[src[src >= 0]] = np.nonzero(src >= 0)[0]
    idx2 = np.full(K1.N, -1, np.int32)
    idx2[pre] = inv[pre]
    mg, mo = m0.copy(), m0.copy()
    ng = ORBmatcher().SearchBySim3(K1, K2, p1, p2, c1, c2, S12, S21, th, mg, idx2)
    no = oracle_lib.OracleMatcher().search_by_sim3(K1, K2, p1, p2, c1, c2, S12, S21, th, mo, idx2)
    assert ng == no
    np.testing.assert_array_equal(mg, mo)
    if scale == 1.0:
        assert no > 100


def test_backend_edges(gpu):
    rng = np.random.default_rng(9)
    KF, cam, pts = sm.synth_fuse_scene(rng, 200, 300)
    m = ORBmatcher()
    n, bi, bd = m.Fuse(KF, cam, pts[:0], 3.0)
    assert n == 0 and len(bi) == 0
    bad = pts.copy()
    bad["flags"] |= 2
    n, bi, bd = m.Fuse(KF, cam, bad, 3.0)
    assert n == 0 and (bi == -1).all() and (bd == -1).all()
    cam2 = sm.synth_kf_camera(rng)
    cam2.Tcw.kind = 7
    with pytest.raises(OrbfeError):
        m.Fuse(KF, cam2, pts, 3.0)


# ---- keyframes with a second camera (NLeft != -1, KannalaBrandt8 stereo) ----
@pytest.mark.parametrize("sides", [(True, True), (True, False), (False, True)], ids=["two_two", "two_one", "one_two"])
@pytest.mark.parametrize("check_ori", [True, False])
def test_search_by_bow_kf_two_cams(gpu, oracle_lib, sides, check_ori):
    """SearchByBoW(KF1, KF2) skips a two-camera keyframe's right indices (ORBmatcher.cc:800-802, 817-819)."""
    rng = np.random.default_rng(21 + sides[0] + 2 * sides[1])
    K1, K2, mp1, mp2, fv1, fv2, _ = sm.synth_two_cam_kf_pair(rng, 600, 560, 200)
    nl1 = K1.nleft if sides[0] else -1
    nl2 = K2.nleft if sides[1] else -1
    for ratio in (0.75, 0.9):
        ng, og = ORBmatcher(ratio, check_ori).SearchByBoWKF(K1.keys, K1.desc, mp1, fv1, K2.keys, K2.desc, mp2, fv2,
                                                            nl1, nl2)
        no, oo = oracle_lib.OracleMatcher(ratio, check_ori).search_by_bow_kf(K1.keys, K1.desc, mp1, fv1, K2.keys,
                                                                              K2.desc, mp2, fv2, nl1, nl2)
        assert ng == no and no > 0
        np.testing.assert_array_equal(og, oo)
        if sides[0]:
            assert (og[K1.nleft:] == -1).all()


@pytest.mark.parametrize("kinds", [(True, True), (False, True), (True, False)], ids=["two_two", "one_two", "two_one"])
@pytest.mark.parametrize("only_stereo", [False, True])
def test_search_for_triangulation_two_cams(gpu, oracle_lib, kinds, only_stereo):
    """SearchForTriangulation with keyframes that have a second camera (bCoarse, as LocalMapping uses
    for inertial maps): kp from mvKeys / mvKeysRight (ORBmatcher.cc:979-1008), bStereo false for them,
    no epipole test when KF1 has one."""
    rng = np.random.default_rng(31 + only_stereo)
    K1, K2, mp1, mp2, fv1, fv2, src = sm.synth_two_cam_kf_pair(rng, 700, 650, 60)

    def single(K):   # the same keypoints as a single-camera pinhole keyframe with stereo uR
        ur = np.where(rng.random(K.N) < 0.6, K.keys["x"] - 10, -1).astype(np.float32)
        return MatchFrame(K.keys, K.desc, K.bounds, K.scale_factors, ur, K.mbf)
    A = K1 if kinds[0] else single(K1)
    B = K2 if kinds[1] else single(K2)
    mp1 = np.where(rng.random(A.N) < 0.4, 5, -1).astype(np.int32)
    mp2 = np.where(rng.random(B.N) < 0.4, 5, -1).astype(np.int32)
    F12 = np.eye(3, dtype=np.float32)
    ep = np.array([256.0, 250.0], np.float32)
    sg = (B.scale_factors * B.scale_factors).astype(np.float32)
    m = ORBmatcher(0.6, True)
    ng, og = m.SearchForTriangulation(A, mp1, fv1, B, mp2, fv2, F12, ep, sg, only_stereo, True)
    no, oo = oracle_lib.OracleMatcher(0.6, True).search_for_triangulation(A, mp1, fv1, B, mp2, fv2, F12, ep, sg,
                                                                           only_stereo, True)
    assert ng == no
    np.testing.assert_array_equal(og, oo)
    assert no > 0 or (only_stereo and (kinds[0] or kinds[1]))
    # the KannalaBrandt8 epipolar test (TriangulateMatches) is the caller's: the bCoarse = false form
    # is orbfe_search_for_triangulation_epi (below); the F12 entry point refuses two-camera keyframes
    with pytest.raises(OrbfeError):
        m.SearchForTriangulation(A, mp1, fv1, B, mp2, fv2, F12, ep, sg, only_stereo, False)


def _epipolar_predicate(salt):
    """A deterministic stand-in for pCamera1->epipolarConstrain(kp1, kp2, ...): passes about 60 % of the
    pairs, decided by a hash of the keypoint pair. The selection logic must call it in an order that
    yields the reference's bestIdx2 whatever the predicate; the real one is the camera model's code,
    which the shim calls unchanged."""
    calls = []

    def epi(i1, i2):
        calls.append((i1, i2))
        h = (i1 * 2654435761 + i2 * 40503 + salt * 97) & 0xFFFFFFFF
        return ((h >> 11) % 5) < 3
    return epi, calls


@pytest.mark.parametrize("kinds", [(True, True), (False, False), (True, False), (False, True)],
                         ids=["two_two", "one_one", "two_one", "one_two"])
@pytest.mark.parametrize("only_stereo,check_ori", [(False, True), (False, False), (True, True)])
def test_search_for_triangulation_epi(gpu, oracle_lib, kinds, only_stereo, check_ori):
    """SearchForTriangulation with bCoarse = false and the epipolar test left to the caller (the
    KannalaBrandt8 keyframes of config 4, LocalMapping.cc:464-466 passes bCoarse = false while
    tracking is healthy): the device lists the gated candidates in (dist, reverse order), the host
    stops at the first that passes; matches12 and nmatches equal the oracle's literal loop
    (ORBmatcher.cc:907-1146) run with the same predicate, which the device form never calls more
    often than the reference does."""
    rng = np.random.default_rng(71 + 2 * only_stereo + check_ori)
    K1, K2, mp1, mp2, fv1, fv2, src = sm.synth_two_cam_kf_pair(rng, 700, 650, 40)

    def single(K):
        ur = np.where(rng.random(K.N) < 0.6, K.keys["x"] - 10, -1).astype(np.float32)
        return MatchFrame(K.keys, K.desc, K.bounds, K.scale_factors, ur, K.mbf)
    A = K1 if kinds[0] else single(K1)
    B = K2 if kinds[1] else single(K2)
    mp1 = np.where(rng.random(A.N) < 0.3, 5, -1).astype(np.int32)
    mp2 = np.where(rng.random(B.N) < 0.3, 5, -1).astype(np.int32)
    ep = np.array([256.0, 250.0], np.float32)
    for salt in (0, 1):
        eg, cg = _epipolar_predicate(salt)
        eo, co = _epipolar_predicate(salt)
        ng, og = ORBmatcher(0.6, check_ori).SearchForTriangulationEpi(A, mp1, fv1, B, mp2, fv2, ep, eg, only_stereo)
        no, oo = oracle_lib.OracleMatcher(0.6, check_ori).search_for_triangulation_epi(A, mp1, fv1, B, mp2, fv2, ep,
                                                                                        eo, only_stereo)
        assert ng == no and (no > 20 or only_stereo)
        np.testing.assert_array_equal(og, oo)
        assert len(cg) <= len(co) and set(cg) <= set(co)


@pytest.mark.parametrize("bright", [False, True], ids=["left", "right"])
@pytest.mark.parametrize("seed,th", [(0, 3.0), (1, 5.0)])
def test_fuse_two_cams(gpu, oracle_lib, seed, th, bright):
    """Fuse(pKF, vpMapPoints, th, bRight) on a KannalaBrandt8 stereo keyframe (ORBmatcher.cc:1148-1298):
    pCamera = mpCamera / mpCamera2, GetRightPose / GetRightCameraCenter, the right grid and
    mvKeysRight, best index NLeft + right index."""
    rng = np.random.default_rng(50 + seed)
    KF = sm.synth_frame_two(rng, 1000, 950)
    cam = sm.synth_camera(rng, rot_deg=20.0)
    rig = sm.synth_rig(cam, True)
    pts = sm.synth_local_map_3d_rig(rng, KF, cam, 8000, two=True)
    kcam = sm.right_kf_camera(cam, rig) if bright else sm.left_kf_camera(cam)
    model = rig.right if bright else rig.left
    ng, big, bdg = ORBmatcher().Fuse(KF, kcam, pts, th, model=model, bRight=bright)
    no, bio, bdo = oracle_lib.OracleMatcher().fuse(KF, kcam, pts, th, model=model, bRight=bright)
    assert ng == no and no > 100
    np.testing.assert_array_equal(big, bio)
    np.testing.assert_array_equal(bdg, bdo)
    hit = big[big >= 0]
    assert ((hit >= KF.nleft) == bright).all()
    # Fuse(pKF, Scw, ...) reads the left camera of the same keyframe
    if not bright:
        ng, big, bdg = ORBmatcher().Fuse(KF, kcam, pts, th, sim3=True, model=model)
        no, bio, bdo = oracle_lib.OracleMatcher().fuse(KF, kcam, pts, th, sim3=True, model=model)
        assert ng == no and no > 0
        np.testing.assert_array_equal(big, bio)
