"""GPU parity: cv::remap INTER_LINEAR (stereo rectification, System.cc:239-240) on the device vs the
CPU oracle, bit-exact, for realistic rectification maps (radial-tangential distortion + rotation),
random maps with out-of-range / negative / exact-integer / huge coordinates, and the batched
device path feeding the extractor."""
import numpy as np
import pytest

from orb_slam3_ros_amd.rectify import rectify_maps, remap_linear, remap_linear_batch
from orb_slam3_ros_amd.synth import synth_image

pytestmark = pytest.mark.gpu


def _rot(deg):
    a = np.deg2rad(deg)
    return np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])


@pytest.mark.parametrize("w,h", [(752, 480), (512, 512), (1241, 376)])
def test_rectify_realistic(gpu, oracle_lib, w, h):
    img = synth_image(w + h, w, h)
    mx, my = rectify_maps(w, h, 458.654, 457.296, w / 2 - 8, h / 2 + 5, (-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05),
                          R=_rot(1.5))
    np.testing.assert_array_equal(remap_linear(img, mx, my), oracle_lib.remap_linear(img, mx, my))


def test_remap_adversarial_maps(gpu, oracle_lib):
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (97, 131), dtype=np.uint8)
    dh, dw = 83, 101
    mx = rng.uniform(-5, 136, (dh, dw)).astype(np.float32)
    my = rng.uniform(-5, 102, (dh, dw)).astype(np.float32)
    mx[::7] = np.round(mx[::7])                       # exact integers: fixed-point cell (0, 0)
    my[::5, ::3] = np.round(my[::5, ::3]) + 0.5
    mx[3, :10] = [-1.0, -0.99, -0.51, -0.5, -0.49, 130.0, 130.49, 130.51, 1e9, -1e9]
    my[4, :6] = [96.0, 96.5, 95.99, -0.5, 1e12, float("nan")]
    np.testing.assert_array_equal(remap_linear(img, mx, my), oracle_lib.remap_linear(img, mx, my))


def test_remap_batch_device(gpu, oracle_lib):
    import torch
    w, h = 752, 480
    imgs = np.stack([synth_image(s, w, h) for s in range(4)])
    mx, my = rectify_maps(w, h, 458.654, 457.296, 367.2, 248.4, (-0.28, 0.07, 2e-4, 1.8e-5), R=_rot(-1.0))
    src = torch.from_numpy(imgs).cuda()
    out = torch.zeros_like(src)
    remap_linear_batch(src, torch.from_numpy(mx).cuda(), torch.from_numpy(my).cuda(), out)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for i in range(4):
        np.testing.assert_array_equal(got[i], oracle_lib.remap_linear(imgs[i], mx, my))


@pytest.mark.parametrize("sw,sh", [(3, 2), (4, 3), (8, 2), (5, 5)])
def test_remap_tiny_sources(gpu, oracle_lib, sw, sh):
    """Sources of < 16 bytes take the guarded byte path (no 8-byte window loads), single and
    batched, including batches that end in a partial image group."""
    import torch
    rng = np.random.default_rng(sw * 10 + sh)
    dh, dw = 6, 9
    mx = rng.uniform(-1.5, sw + 0.5, (dh, dw)).astype(np.float32)
    my = rng.uniform(-1.5, sh + 0.5, (dh, dw)).astype(np.float32)
    imgs = rng.integers(0, 256, (11, sh, sw), dtype=np.uint8)
    np.testing.assert_array_equal(remap_linear(imgs[0], mx, my), oracle_lib.remap_linear(imgs[0], mx, my))
    src = torch.from_numpy(imgs).cuda()
    out = torch.zeros((11, dh, dw), dtype=torch.uint8, device="cuda")
    remap_linear_batch(src, torch.from_numpy(mx).cuda(), torch.from_numpy(my).cuda(), out)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for i in range(11):
        np.testing.assert_array_equal(got[i], oracle_lib.remap_linear(imgs[i], mx, my))


@pytest.mark.parametrize("dist", [
    (-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05),            # EuRoC cam0 (radial-tangential)
    (-0.28, 0.07, 2e-4, 1.8e-5, 0.01),                                 # + k3
    (0.5, -0.3, 1e-3, -2e-3, 0.1, 0.4, -0.2, 0.05),                    # rational model
    (-1.5, 0.9, 0.01, 0.01),                                           # strong: icdist < 0 near corners
])
def test_undistort_points(gpu, oracle_lib, dist):
    from orb_slam3_ros_amd.rectify import undistort_points
    rng = np.random.default_rng(len(dist))
    K = (458.654, 457.296, 367.215, 248.375)
    pts = np.stack([rng.uniform(-20, 772, 5000), rng.uniform(-20, 500, 5000)], 1).astype(np.float32)
    pts[:4] = [[0, 0], [751, 479], [K[2], K[3]], [367.2151, 248.3749]]
    g = undistort_points(pts, K, np.array(dist, np.float32))
    o = oracle_lib.undistort_points(pts, K, np.array(dist, np.float32))
    np.testing.assert_array_equal(g.view(np.uint32), o.view(np.uint32))


def test_remap_batch_alternating_buffer_sets(gpu, oracle_lib):
    """The device pointer-table ring (4 slots keyed by the pointers): two double-buffered sets
    alternated without host syncs, then six sets (more than the ring holds) cycled, each launch
    checked against the oracle; tables re-uploaded asynchronously must never be read stale."""
    import torch
    w, h, n = 160, 120, 3
    mx, my = rectify_maps(w, h, 150.0, 150.0, 80.0, 60.0, (-0.2, 0.05, 1e-4, 1e-5), R=_rot(2.0))
    dmx, dmy = torch.from_numpy(mx).cuda(), torch.from_numpy(my).cuda()
    imgs = [np.stack([synth_image(100 * k + i, w, h) for i in range(n)]) for k in range(6)]
    want = [[oracle_lib.remap_linear(imgs[k][i], mx, my) for i in range(n)] for k in range(6)]
    srcs = [torch.from_numpy(im).cuda() for im in imgs]
    for order in ([0, 1] * 4, [0, 1, 2, 3, 4, 5, 0, 5, 1, 4, 2, 3]):
        outs = []
        for k in order:   # each launch writes a fresh output: every result stays checkable
            out = torch.zeros((n, h, w), dtype=torch.uint8, device="cuda")
            remap_linear_batch(srcs[k], dmx, dmy, out)
            outs.append((k, out))
        torch.cuda.synchronize()
        for k, out in outs:
            got = out.cpu().numpy()
            for i in range(n):
                np.testing.assert_array_equal(got[i], want[k][i])


def test_remap_batch_pitched_source(gpu, oracle_lib):
    """Sources with a row pitch above the width (padding filled with 255) and a buffer that ends at
    the last row's width: the fast path's window stays inside the image columns."""
    import torch
    w, h, pitch, n = 200, 90, 256, 2
    mx, my = rectify_maps(w, h, 180.0, 180.0, 100.0, 45.0, (-0.25, 0.06, 2e-4, -1e-4), R=_rot(-2.0))
    imgs = np.stack([synth_image(7 + i, w, h) for i in range(n)])
    flat = torch.full((n * h * pitch - (pitch - w),), 255, dtype=torch.uint8, device="cuda")
    src = flat.as_strided((n, h, w), (h * pitch, pitch, 1))
    src.copy_(torch.from_numpy(imgs).cuda())
    out = torch.zeros((n, h, w), dtype=torch.uint8, device="cuda")
    remap_linear_batch(src, torch.from_numpy(mx).cuda(), torch.from_numpy(my).cuda(), out)
    torch.cuda.synchronize()
    for i in range(n):
        np.testing.assert_array_equal(out[i].cpu().numpy(), oracle_lib.remap_linear(imgs[i], mx, my))


def test_remap_batch_two_streams(gpu, oracle_lib):
    """The pointer-table ring used from two streams: six fixed (source, output) sets cycled over two
    alternating streams (more sets than ring slots, so slots are refilled while the other stream may
    still read them, and hits come on another stream than the upload). Each launch is preceded on
    its own stream by zeroing its output, so a launch that read a stale or partly written table
    leaves its set's output zero (or writes another set's): every final output is checked."""
    import torch
    w, h, n = 160, 120, 2
    mx, my = rectify_maps(w, h, 150.0, 150.0, 80.0, 60.0, (-0.2, 0.05, 1e-4, 1e-5), R=_rot(1.0))
    dmx, dmy = torch.from_numpy(mx).cuda(), torch.from_numpy(my).cuda()
    imgs = [np.stack([synth_image(300 + 10 * k + i, w, h) for i in range(n)]) for k in range(6)]
    srcs = [torch.from_numpy(im).cuda() for im in imgs]
    outs = [torch.zeros((n, h, w), dtype=torch.uint8, device="cuda") for _ in range(6)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    order = [0, 1, 2, 3, 4, 5, 0, 0, 5, 1, 4, 2, 3, 3, 1, 0, 2, 4, 5, 1]
    for j, k in enumerate(order):
        s = streams[j & 1]
        with torch.cuda.stream(s):
            outs[k].zero_()
            remap_linear_batch(srcs[k], dmx, dmy, outs[k], stream=s.cuda_stream)
    torch.cuda.synchronize()
    for k in range(6):
        got = outs[k].cpu().numpy()
        for i in range(n):
            np.testing.assert_array_equal(got[i], oracle_lib.remap_linear(imgs[k][i], mx, my))
