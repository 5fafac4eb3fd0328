"""CPU: the oracle against its committed golden fixtures (regression pin; see make_golden.py) and
known-answer tests of the primitives restated from OpenCV 4.2."""
import hashlib
import os

import numpy as np
import pytest

from orb_slam3_ros_amd.synth import synth_image, synth_stereo

GOLD = os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.npz")
CASES = {"euroc_mono": 1, "euroc_stereo_l": 2, "kitti": 3, "tumvi": 4}


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD, allow_pickle=False)


@pytest.mark.parametrize("name", list(CASES))
def test_extractor_golden(name, gold, oracle_lib):
    w, h, nf, lap0, lap1 = gold[name + "_meta"].tolist()
    img = synth_image(CASES[name], w, h)
    assert hashlib.sha256(img.tobytes()).digest() == gold[name + "_img_sha"].tobytes(), "synthetic generator drifted"
    ex = oracle_lib.OracleExtractor(nf, 1.2, 8, 20, 7)
    mono, kp, desc = ex(img, (lap0, lap1))
    assert mono == int(gold[name + "_mono"][0])
    assert np.array_equal(kp.view(np.uint8).reshape(len(kp), 28), gold[name + "_kp"])
    assert np.array_equal(desc, gold[name + "_desc"])
    for l in range(8):
        p = ex.pyramid_level(l)
        assert [int(p.astype(np.int64).sum()), p.shape[0], p.shape[1]] == gold[f"{name}_pyr{l}_sum"].tolist()


def test_stereo_golden(gold, oracle_lib):
    left, right = synth_stereo(5)
    assert hashlib.sha256(left.tobytes() + right.tobytes()).digest() == gold["stereo_img_sha"].tobytes()
    el, er = oracle_lib.OracleExtractor(1200, 1.2, 8, 20, 7), oracle_lib.OracleExtractor(1200, 1.2, 8, 20, 7)
    _, kl, dl = el(left)
    _, kr, dr = er(right)
    ur, dp, nm = oracle_lib.stereo_match(el, er, kl, dl, kr, dr, 0.110078 * 435.2, 435.2)
    assert nm == int(gold["stereo_nmatch"][0])
    assert np.array_equal(ur.view(np.uint32), gold["stereo_uright"].view(np.uint32))
    assert np.array_equal(dp.view(np.uint32), gold["stereo_depth"].view(np.uint32))
    good = ur >= 0
    assert good.sum() > 0.3 * len(kl)
    assert np.all(ur[good] <= kl["x"][good] + 1e-3)


# ---- known-answer tests of the restated OpenCV primitives ----
def _fast(oracle_lib, roi, th):
    import ctypes
    L = oracle_lib.lib()
    roi = np.ascontiguousarray(roi, np.uint8)
    out = np.zeros(4096, oracle_lib.KEYPOINT_DTYPE)
    n = L.oro_fast(roi.ctypes.data, roi.shape[1], roi.shape[0], roi.shape[1], th, out.ctypes.data, 4096)
    return out[:n]


def test_fast_isolated_bright_pixel(oracle_lib):
    roi = np.full((15, 15), 50, np.uint8)
    roi[7, 7] = 200
    kp = _fast(oracle_lib, roi, 20)
    assert len(kp) == 1 and kp["x"][0] == 7 and kp["y"][0] == 7
    # every ring pixel is 150 darker: M = 150, score = max(th, M) - 1
    assert kp["response"][0] == 149.0 and kp["size"][0] == 7.0 and kp["angle"][0] == -1.0


def test_fast_threshold_is_strict(oracle_lib):
    roi = np.full((15, 15), 100, np.uint8)
    roi[7, 7] = 120          # contrast exactly 20: not > 20
    assert len(_fast(oracle_lib, roi, 20)) == 0
    roi[7, 7] = 121
    kp = _fast(oracle_lib, roi, 20)
    assert len(kp) == 1 and kp["response"][0] == 20.0


def test_fast_scan_border(oracle_lib):
    roi = np.full((10, 10), 50, np.uint8)
    roi[2, 5] = 250          # row 2 is outside rows 3..rows-4
    roi[5, 6] = 250          # col 6 == cols-4 is inside
    kp = _fast(oracle_lib, roi, 20)
    assert [(int(k["x"]), int(k["y"])) for k in kp] == [(6, 5)]


def test_fast_nms_keeps_strict_maximum(oracle_lib):
    roi = np.full((15, 15), 50, np.uint8)
    roi[7, 7] = 200
    roi[7, 8] = 199
    kp = _fast(oracle_lib, roi, 20)
    assert [(int(k["x"]), int(k["y"])) for k in kp] == [(7, 7)]


def test_fast_atan2_quadrants(oracle_lib):
    L = oracle_lib.lib()
    assert L.oro_fast_atan2(0.0, 1.0) == 0.0
    assert abs(L.oro_fast_atan2(1.0, 0.0) - 90.0) < 1e-4
    assert abs(L.oro_fast_atan2(0.0, -1.0) - 180.0) < 1e-4
    assert abs(L.oro_fast_atan2(-1.0, 0.0) - 270.0) < 1e-4
    assert abs(L.oro_fast_atan2(1.0, 1.0) - 45.0) < 0.01


def test_blur_constant_and_kernel_sums(oracle_lib):
    L = oracle_lib.lib()
    img = np.full((20, 30), 77, np.uint8)
    out = np.zeros_like(img)
    for variant in (0, 1):
        L.oro_blur(img.ctypes.data, 30, 20, out.ctypes.data, variant)
        # ED kernel sums to 256 -> exact; per-tap kernel sums to 257 -> (77*257*257 + 2^15) >> 16
        expect = 77 if variant == 0 else (77 * 257 * 257 + 32768) >> 16
        assert np.all(out == expect)


def test_resize_identity_and_size(oracle_lib):
    L = oracle_lib.lib()
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (40, 60), dtype=np.uint8)
    out = np.zeros((40, 60), np.uint8)
    L.oro_resize(img.ctypes.data, 60, 40, out.ctypes.data, 60, 40, 16)
    assert np.array_equal(img, out)
    flat = np.full((48, 60), 200, np.uint8)
    small = np.zeros((40, 50), np.uint8)
    L.oro_resize(flat.ctypes.data, 60, 48, small.ctypes.data, 50, 40, 16)
    assert np.all(small == 200)


def test_hamming(oracle_lib):
    L = oracle_lib.lib()
    a = np.zeros(32, np.uint8)
    b = np.full(32, 255, np.uint8)
    assert L.oro_hamming(a.ctypes.data, b.ctypes.data) == 256
    b[:] = 0
    b[5] = 0b1011
    assert L.oro_hamming(a.ctypes.data, b.ctypes.data) == 3
