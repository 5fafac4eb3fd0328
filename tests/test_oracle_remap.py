"""CPU: the cv::remap oracle's fixed-point table equals the closed form the HIP kernel uses, and
remap semantics on known answers (identity map, integer shifts, constant border)."""
import numpy as np

from orb_slam3_ros_amd.rectify import rectify_maps


def test_bilinear_tab_closed_form(oracle_lib):
    t = oracle_lib.remap_bilinear_tab().astype(np.int64)
    for a in range(1024):
        ay, ax = divmod(a, 32)
        if a == 0:
            exp = [32767, 0, 0, 1]   # 32768 saturates; initInterTab2D adds the deficit to w11
        else:
            exp = [(32 - ay) * (32 - ax) * 32, (32 - ay) * ax * 32, ay * (32 - ax) * 32, ay * ax * 32]
        assert t[a].tolist() == exp, a
        assert t[a].sum() == 32768


def test_remap_identity_shift_border(oracle_lib):
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (40, 50), dtype=np.uint8)
    v, u = np.mgrid[0:40, 0:50].astype(np.float32)
    assert np.array_equal(oracle_lib.remap_linear(img, u, v), img)
    out = oracle_lib.remap_linear(img, u + 3, v - 2)
    assert np.array_equal(out[2:, :47], img[:38, 3:])
    assert (out[:1, :] == 0).all() and (out[:, 49:] == 0).all()   # footprint fully outside: 0
    half = oracle_lib.remap_linear(img, u + 0.5, v)
    ref = (img[:, :-1].astype(np.int32) * 16384 + img[:, 1:].astype(np.int32) * 16384 + 16384) >> 15
    assert np.array_equal(half[:, :-1], ref)


def test_rectify_maps_identity():
    mx, my = rectify_maps(64, 48, 50.0, 50.0, 32.0, 24.0)
    v, u = np.mgrid[0:48, 0:64].astype(np.float32)
    assert np.allclose(mx, u, atol=1e-4) and np.allclose(my, v, atol=1e-4)


def test_undistort_points_oracle_properties(oracle_lib):
    """Zero distortion is the identity; with distortion, re-distorting the result lands back on
    the input to well under a pixel (5 fixed-point iterations)."""
    K = (458.654, 457.296, 367.215, 248.375)
    rng = np.random.default_rng(2)
    pts = np.stack([rng.uniform(0, 752, 500), rng.uniform(0, 480, 500)], 1).astype(np.float32)
    out0 = oracle_lib.undistort_points(pts, K, np.zeros(4, np.float32))
    assert np.allclose(out0, pts, atol=1e-3)
    D = np.array([-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05], np.float32)
    und = oracle_lib.undistort_points(pts, K, D).astype(np.float64)
    x = (und[:, 0] - K[2]) / K[0]
    y = (und[:, 1] - K[3]) / K[1]
    r2 = x * x + y * y
    k1, k2, p1, p2 = D.astype(np.float64)
    kr = 1 + (k1 + k2 * r2) * r2
    xd = x * kr + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * kr + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    back = np.stack([xd * K[0] + K[2], yd * K[1] + K[3]], 1)
    centre = np.linalg.norm(pts - [K[2], K[3]], axis=1) < 250
    assert np.abs(back - pts)[centre].max() < 0.5
