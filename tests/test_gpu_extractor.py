"""GPU parity: the HIP ORB extractor (through the C-ABI) against the CPU oracle, bit-exact.

Covers every intermediate the reference materialises (pyramid levels, per-cell FAST keys,
DistributeOctTree output) and the final operator() outputs (keypoints incl. order, descriptors,
monoIndex) for the BASELINE configs' image sizes and feature budgets, lapping areas {0,0},
{0,1000} and {0,511}, and edge inputs (flat image, tiny image, noise only).
"""
import numpy as np
import pytest

from orb_slam3_ros_amd.synth import synth_image, synth_stereo

pytestmark = pytest.mark.gpu

CONFIGS = [  # (w, h, nfeatures) from BASELINE.json configs 1-4
    (752, 480, 1000),
    (752, 480, 1200),
    (1241, 376, 2000),
    (512, 512, 1000),
]


def _unpack(keys):
    keys = np.asarray(keys, np.uint32)
    return keys & 0xFFF, (keys >> 12) & 0xFFF, keys >> 24


def _gpu_cell_keys(ext, level, ncell, cell_cap):
    import ctypes
    lib = ext._lib
    cnt = np.zeros(ncell, np.int32)
    lib.orbfe_debug_copy(ext.handle, 0, 0, level, cnt.ctypes.data, cnt.nbytes)
    slots = np.zeros(ncell * cell_cap, np.uint32)
    lib.orbfe_debug_copy(ext.handle, 1, 0, level, slots.ctypes.data, slots.nbytes)
    out = [slots[c * cell_cap: c * cell_cap + cnt[c]] for c in range(ncell)]
    return np.concatenate(out) if out else np.zeros(0, np.uint32)


def _gpu_octree(ext, level):
    info = np.zeros(4, np.int32)
    ext._lib.orbfe_debug_copy(ext.handle, 3, 0, level, info.ctypes.data, 16)
    keys = np.zeros(max(info[0], 1), np.uint32)
    ext._lib.orbfe_debug_copy(ext.handle, 2, 0, level, keys.ctypes.data, keys.nbytes)
    return keys[: info[0]], info


def _cell_geom(w, h):
    width, height = np.float32(w - 32), np.float32(h - 32)
    ncols, nrows = int(width / np.float32(35)), int(height / np.float32(35))
    wc, hc = int(np.ceil(width / np.float32(ncols))), int(np.ceil(height / np.float32(nrows)))
    return ncols * nrows, ((wc + 1) // 2) * ((hc + 1) // 2)


def _compare_extract(img, nfeat, lap, oracle_lib, check_stages=True):
    from orb_slam3_ros_amd.extractor import ORBextractor
    ext = ORBextractor(nfeat, 1.2, 8, 20, 7)
    ora = oracle_lib.OracleExtractor(nfeat, 1.2, 8, 20, 7)
    mono_g, kp_g, d_g = ext(img, None, lap)
    mono_o, kp_o, d_o = ora(img, lap)
    if check_stages:
        for l in range(8):
            pg, po = ext.pyramid_level(l), ora.pyramid_level(l)
            assert pg.shape == po.shape, f"level {l} size"
            bad = np.argwhere(pg != po)
            assert bad.size == 0, f"pyramid level {l}: {len(bad)} px differ, first {bad[:3].tolist()}"
        for l in range(8):
            raw_o = ora.debug_keys(l, 0)
            ncell, cap = _cell_geom(*pg.shape[::-1]) if False else _cell_geom(*ora.pyramid_level(l).shape[::-1])
            raw_g = _gpu_cell_keys(ext, l, ncell, cap)
            gx, gy, gs = _unpack(raw_g)
            assert len(raw_g) == len(raw_o), f"level {l}: raw FAST count gpu {len(raw_g)} vs oracle {len(raw_o)}"
            assert np.array_equal(gx, raw_o["x"].astype(np.uint32)), f"level {l} raw x"
            assert np.array_equal(gy, raw_o["y"].astype(np.uint32)), f"level {l} raw y"
            assert np.array_equal(gs, raw_o["response"].astype(np.uint32)), f"level {l} raw score"
            oct_g, info = _gpu_octree(ext, l)
            oct_o = ora.debug_keys(l, 1)
            ox, oy, os_ = _unpack(oct_g)
            assert len(oct_g) == len(oct_o), f"level {l}: octree count gpu {len(oct_g)} vs oracle {len(oct_o)}"
            assert np.array_equal(ox, oct_o["x"].astype(np.uint32)), f"level {l} octree x order"
            assert np.array_equal(oy, oct_o["y"].astype(np.uint32)), f"level {l} octree y order"
    assert mono_g == mono_o
    assert len(kp_g) == len(kp_o)
    for f in ("x", "y", "size", "response", "octave", "class_id"):
        assert np.array_equal(kp_g[f], kp_o[f]), f"keypoint field {f}"
    bad = np.nonzero(kp_g["angle"].view(np.uint32) != kp_o["angle"].view(np.uint32))[0]
    assert bad.size == 0, f"angle mismatch at {bad[:5].tolist()}: {kp_g['angle'][bad[:5]]} vs {kp_o['angle'][bad[:5]]}"
    rows = np.nonzero((d_g != d_o).any(axis=1))[0]
    assert rows.size == 0, f"{rows.size} descriptor rows differ, first {rows[:5].tolist()}"
    ext.close()
    return len(kp_g)


@pytest.mark.parametrize("w,h,nfeat", CONFIGS)
def test_extract_matches_oracle(w, h, nfeat, gpu, oracle_lib):
    """Every intermediate: pyramid levels, per-cell FAST keys, octree output, final outputs."""
    img = synth_image(100 + w, w, h)
    n = _compare_extract(img, nfeat, (0, 0), oracle_lib)
    assert n >= nfeat * 0.9


@pytest.mark.parametrize("lap", [(0, 1000), (0, 511), (200, 400)])
def test_lapping_reorder(lap, gpu, oracle_lib):
    img = synth_image(7, 752, 480)
    _compare_extract(img, 1000, lap, oracle_lib, check_stages=False)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_more_seeds(seed, gpu, oracle_lib):
    img = synth_image(seed, 752, 480)
    _compare_extract(img, 1000, (0, 1000), oracle_lib, check_stages=False)


def test_flat_and_noise_images(gpu, oracle_lib):
    flat = np.full((480, 752), 128, np.uint8)
    _compare_extract(flat, 1000, (0, 0), oracle_lib, check_stages=False)
    rng = np.random.default_rng(5)
    noise = rng.integers(0, 256, (480, 752), dtype=np.uint8)
    _compare_extract(noise, 1000, (0, 0), oracle_lib)
    grad = np.tile(np.arange(752, dtype=np.uint8), (480, 1))
    _compare_extract(grad, 1000, (0, 0), oracle_lib, check_stages=False)


def test_small_image(gpu, oracle_lib):
    img = synth_image(11, 400, 300)
    _compare_extract(img, 500, (0, 0), oracle_lib)


def test_large_cells(gpu, oracle_lib):
    # 362x362: the top levels have a single 69x69 FAST cell (W/35 just below 2), which exceeds
    # the kernel's register prefetch window and exercises its direct-load path
    img = synth_image(12, 362, 362)
    _compare_extract(img, 1000, (0, 0), oracle_lib)


def test_mono_init_5000(gpu, oracle_lib):
    # Tracking's mpIniORBextractor uses 5*nFeatures while uninitialised (Tracking.cc:637,1622)
    img = synth_image(21, 752, 480)
    _compare_extract(img, 5000, (0, 1000), oracle_lib, check_stages=False)


def test_empty_image(gpu):
    from orb_slam3_ros_amd.extractor import ORBextractor
    ext = ORBextractor(1000, 1.2, 8, 20, 7)
    mono, kp, d = ext(np.zeros((0, 0), np.uint8))
    assert mono == -1 and len(kp) == 0


@pytest.mark.parametrize("nfeat", [1200, 2500])
def test_stereo_matches_oracle(gpu, oracle_lib, nfeat):
    """ComputeStereoMatches bit-exact; 2500 features puts more than 2048 keypoints in an image
    (the stereo kernels have no sort-size limit, only their LDS)."""
    from orb_slam3_ros_amd.extractor import ORBextractor, compute_stereo_matches
    left, right = synth_stereo(3, 752, 480)
    el, er = ORBextractor(nfeat, 1.2, 8, 20, 7), ORBextractor(nfeat, 1.2, 8, 20, 7)
    ol, orr = oracle_lib.OracleExtractor(nfeat, 1.2, 8, 20, 7), oracle_lib.OracleExtractor(nfeat, 1.2, 8, 20, 7)
    _, kl, dl = el(left, None, (0, 0))
    _, kr, dr = er(right, None, (0, 0))
    _, okl, odl = ol(left)
    _, okr, odr = orr(right)
    assert np.array_equal(dl, odl) and np.array_equal(dr, odr)
    bf, fx = 0.110078 * 435.2, 435.2
    ur, dp, nm = compute_stereo_matches(el, er, bf, fx, len(kl))
    our, odp, onm = oracle_lib.stereo_match(ol, orr, okl, odl, okr, odr, bf, fx)
    assert nm == onm
    assert np.array_equal(ur.view(np.uint32), our.view(np.uint32)), np.nonzero(ur != our)[0][:10]
    assert np.array_equal(dp.view(np.uint32), odp.view(np.uint32))
    assert (ur >= 0).sum() > 0.3 * len(kl)


def test_stereo_matches_tall_image(gpu, oracle_lib):
    """Images taller than 1983 rows take k_stereo's bitonic-sort / binary-search ordering of the
    right records (the row-count table of the counting sort no longer fits): bit-exact too."""
    from orb_slam3_ros_amd.extractor import ORBextractor, compute_stereo_matches
    left, right = synth_stereo(5, 1152, 2048)   # width >= height / 2: the octree needs nIni >= 1
    el, er = ORBextractor(1500, 1.2, 8, 20, 7), ORBextractor(1500, 1.2, 8, 20, 7)
    ol, orr = oracle_lib.OracleExtractor(1500, 1.2, 8, 20, 7), oracle_lib.OracleExtractor(1500, 1.2, 8, 20, 7)
    _, kl, dl = el(left, None, (0, 0))
    _, kr, dr = er(right, None, (0, 0))
    _, okl, odl = ol(left)
    _, okr, odr = orr(right)
    assert np.array_equal(kl.view(np.uint8), okl.view(np.uint8)) and np.array_equal(dr, odr)
    bf, fx = 0.110078 * 435.2, 435.2
    ur, dp, nm = compute_stereo_matches(el, er, bf, fx, len(kl))
    our, odp, onm = oracle_lib.stereo_match(ol, orr, okl, odl, okr, odr, bf, fx)
    assert nm == onm
    assert np.array_equal(ur.view(np.uint32), our.view(np.uint32)), np.nonzero(ur != our)[0][:10]
    assert np.array_equal(dp.view(np.uint32), odp.view(np.uint32))
    assert (ur >= 0).sum() > 0.3 * len(kl)


def test_host_call_sequence(gpu, oracle_lib):
    """A sequence of orbfe_extract calls on one handle, as Tracking makes them (one-image output block,
    single result copy): every call stays bit-exact across image changes, a lapping-area change, a
    batch call on the same handle in between (the next host call re-uploads the batch description)
    and an OpenCV-model round trip (buffers rebuilt); the pyramid getter reads the last call's
    levels."""
    import ctypes

    import torch
    from orb_slam3_ros_amd.extractor import ORBextractor
    ext = ORBextractor(1000, 1.2, 8, 20, 7)
    ora = oracle_lib.OracleExtractor(1000, 1.2, 8, 20, 7)

    def check(img, lap):
        mono_g, kp_g, d_g = ext(img, None, lap)
        mono_o, kp_o, d_o = ora(img, lap)
        assert mono_g == mono_o and len(kp_g) == len(kp_o)
        assert np.array_equal(kp_g.view(np.uint8), kp_o.view(np.uint8))
        assert np.array_equal(d_g, d_o)

    seeds = iter(range(300, 400))
    for lap in [(0, 0)] * 4 + [(0, 1000)] * 3:
        check(synth_image(next(seeds), 752, 480), lap)
    # the last call's pyramid, as Frame reads mvImagePyramid
    img = synth_image(next(seeds), 752, 480)
    check(img, (0, 1000))
    for l in (0, 3, 7):
        assert np.array_equal(ext.pyramid_level(l), ora.pyramid_level(l))
    # a batch call on the same handle between two host calls
    batch = torch.from_numpy(np.stack([synth_image(next(seeds), 752, 480) for _ in range(2)])).cuda()
    ptrs = (ctypes.c_void_p * 2)(*(batch[i].data_ptr() for i in range(2)))
    assert ext._lib.orbfe_extract_batch(ext.handle, 2, ptrs, 752, 480, 752, 0, 1000, None) == 0
    torch.cuda.synchronize()
    for _ in range(3):
        check(synth_image(next(seeds), 752, 480), (0, 1000))
    # buffers rebuilt by a model change and back
    for lanes in (8, 16):
        ext.set_opencv_model(lanes, 0)
        ora._l.oro_set_model(ora.h, lanes, 0)
        for _ in range(3):
            check(synth_image(next(seeds), 752, 480), (0, 1000))
    ext.close()


@pytest.mark.parametrize("nfeat,size", [(1000, (752, 480)), (2000, (1241, 376))])
def test_frame_stereo_entry(gpu, oracle_lib, nfeat, size):
    """orbfe_frame_stereo (Frame::Frame(stereo), Frame.cc:101-141, in one call) against the oracle's
    two extractions + ComputeStereoMatches: keypoints, descriptors, monoIndex, uR / depth bits and
    the match count, over a seeded sequence of frames on the same handles (one handle reused after
    a host orbfe_extract call in between, and the right image's pyramid read back from the left
    handle's image 1)."""
    from orb_slam3_ros_amd.extractor import ORBextractor, frame_stereo
    from orb_slam3_ros_amd.synth import synth_stereo_sequence
    w, h = size
    bf, fx = 0.110078 * 458.654, 458.654
    el, er = ORBextractor(nfeat, 1.2, 8, 20, 7), ORBextractor(nfeat, 1.2, 8, 20, 7)
    seq = synth_stereo_sequence(11, 3, w, h)
    for k, (left, right) in enumerate(seq):
        if k == 1:   # a plain host call on the left handle in between
            el(left, None, (0, 0))
        (ml, kl, dl), (mr, kr, dr), ur, dp, nm = frame_stereo(el, er, left, right, bf, fx)
        ol, orr = oracle_lib.OracleExtractor(nfeat, 1.2, 8, 20, 7), oracle_lib.OracleExtractor(nfeat, 1.2, 8, 20, 7)
        oml, okl, odl = ol(left)
        omr, okr, odr = orr(right)
        assert (ml, mr) == (oml, omr)
        assert np.array_equal(kl.view(np.uint8), okl.view(np.uint8)) and np.array_equal(dl, odl)
        assert np.array_equal(kr.view(np.uint8), okr.view(np.uint8)) and np.array_equal(dr, odr)
        our, odp, onm = oracle_lib.stereo_match(ol, orr, okl, odl, okr, odr, bf, fx)
        assert nm == onm
        assert np.array_equal(ur.view(np.uint32), our.view(np.uint32)), np.nonzero(ur != our)[0][:10]
        assert np.array_equal(dp.view(np.uint32), odp.view(np.uint32))
        assert (ur >= 0).sum() > 0.3 * len(kl)
        for lv in (0, 3, 7):
            assert np.array_equal(el.pyramid_level(lv, image=1), orr.pyramid_level(lv))


def test_frame_stereo_rejects_mismatched_handles(gpu):
    from orb_slam3_ros_amd import _lib
    from orb_slam3_ros_amd.extractor import ORBextractor, frame_stereo
    left, right = synth_stereo(4, 752, 480)
    el, er = ORBextractor(1000, 1.2, 8, 20, 7), ORBextractor(1200, 1.2, 8, 20, 7)
    with pytest.raises(_lib.OrbfeError):
        frame_stereo(el, er, left, right, 50.0, 458.0)


def test_frame_device_view_searches(gpu):
    """Tracking's searches on the current frame read it in HBM (orbfe_frame_device_view of the last
    orbfe_frame_stereo): SearchByProjection(F, local map) and SearchByProjection(CurrentFrame,
    LastFrame) give the same slots and counts through the device view as through the host copy; a
    stale id (the handle extracted since) and a shape outside the one-workgroup path are refused."""
    from orb_slam3_ros_amd import _lib
    from orb_slam3_ros_amd import synth_match as sm
    from orb_slam3_ros_amd.extractor import ORBextractor, frame_stereo
    from orb_slam3_ros_amd.matcher import MatchFrame, ORBmatcher, current_frame_view
    from orb_slam3_ros_amd.synth import synth_stereo
    bf, fx = 0.110078 * 458.654, 458.654
    el, er = ORBextractor(1000, 1.2, 8, 20, 7), ORBextractor(1000, 1.2, 8, 20, 7)
    left, right = synth_stereo(5, 752, 480)
    (ml, kl, dl), _, ur, _, _ = frame_stereo(el, er, left, right, bf, fx)
    lib = _lib.load()
    fid = lib.orbfe_extractor_frame_id(el.handle)
    F = MatchFrame(kl, dl, (0.0, 752.0, 0.0, 480.0), np.asarray(el.GetScaleFactors(), np.float32), ur, bf)
    V = current_frame_view(F, el, fid)
    assert V is not None and V.N == F.N
    rng = np.random.default_rng(3)
    mps = sm.synth_local_map(rng, F, 1500)
    mvp0, obs = sm.initial_slots(rng, F.N)
    m = ORBmatcher(0.8)
    for th in (1.0, 3.0):
        a, b = mvp0.copy(), mvp0.copy()
        assert m.SearchByProjectionLocalMap(V, a, obs, mps, th) == m.SearchByProjectionLocalMap(F, b, obs, mps, th)
        np.testing.assert_array_equal(a, b)
    pts = sm.synth_proj_points(rng, F, 900)
    for fwd, bwd in ((0, 0), (1, 0)):
        a, b = mvp0.copy(), mvp0.copy()
        ga = m.SearchByProjectionLastFrame(V, a, obs, pts, 7.0, fwd, bwd)
        gb = m.SearchByProjectionLastFrame(F, b, obs, pts, 7.0, fwd, bwd)
        assert ga == gb
        np.testing.assert_array_equal(a, b)
    # the device-projected last-frame search (the shim's form) on the view as well
    from orb_slam3_ros_amd.matcher import CameraModel, Pose
    model = CameraModel.make("pinhole", fx, 457.296, 367.215, 248.375)
    R, t = sm.synth_pose(rng)
    lp = sm.synth_last_points(rng, F, model, R, t, 900)
    a, b = mvp0.copy(), mvp0.copy()
    ga = m.SearchByProjectionLastFramePose(V, a, obs, lp, Pose.se3(R, t), model, 7.0, False, False)
    gb = m.SearchByProjectionLastFramePose(F, b, obs, lp, Pose.se3(R, t), model, 7.0, False, False)
    assert ga == gb and ga > 0
    np.testing.assert_array_equal(a, b)
    big = sm.synth_local_map(rng, F, 5000)   # > 2048 queries: not the one-workgroup path
    with pytest.raises(_lib.OrbfeError):
        m.SearchByProjectionLocalMap(V, mvp0.copy(), obs, big, 1.0)
    el(left, None, (0, 0))   # the handle extracts again: the view is stale
    assert current_frame_view(F, el, fid) is None


@pytest.mark.parametrize("lap", [(0, 511), (100, 400)])
def test_frame_fisheye_entry(gpu, oracle_lib, lap):
    """orbfe_frame_fisheye (Frame(stereo, KannalaBrandt8) up to its descriptor stage, Frame.cc:1034-1151,
    in one call) against the oracle's two extractions with the same vLappingArea + knnMatch(k=2) +
    ratio 0.7 over the lapping rows: keypoints, descriptors, monoIndex, the l2r candidates and their
    count, over a seeded sequence on the same handles."""
    from orb_slam3_ros_amd.extractor import ORBextractor, frame_fisheye
    el, er = ORBextractor(1000, 1.2, 8, 20, 7), ORBextractor(1000, 1.2, 8, 20, 7)
    for seed in (31, 32, 33):
        left, right = synth_stereo(seed, 512, 512)
        (ml, kl, dl), (mr, kr, dr), l2r, dist, ng = frame_fisheye(el, er, left, right, lap, 0.7)
        ol, orr = oracle_lib.OracleExtractor(1000, 1.2, 8, 20, 7), oracle_lib.OracleExtractor(1000, 1.2, 8, 20, 7)
        oml, okl, odl = ol(left, lap)
        omr, okr, odr = orr(right, lap)
        assert (ml, mr) == (oml, omr)
        assert np.array_equal(kl.view(np.uint8), okl.view(np.uint8)) and np.array_equal(dl, odl)
        assert np.array_equal(kr.view(np.uint8), okr.view(np.uint8)) and np.array_equal(dr, odr)
        g, t, d = oracle_lib.stereo_knn_ratio(odl[oml:], odr[omr:], 0.7)
        exp, expd = np.full(len(okl), -1, np.int32), np.full(len(okl), -1, np.int32)
        exp[oml:][t >= 0] = t[t >= 0] + omr
        expd[oml:][t >= 0] = d[t >= 0]
        assert ng == g and g > 50
        np.testing.assert_array_equal(l2r, exp)
        np.testing.assert_array_equal(dist, expd)
        ol.close()
        orr.close()

