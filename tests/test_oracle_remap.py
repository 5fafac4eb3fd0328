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
