"""The compiled C++ consumer of the C-ABI (tests/native/capi_frontend.cpp: include/orbfe.h only, linked
against liborbfe.so, mirroring shim/ORBextractor_orbfe.cc + shim/ORBmatcher_orbfe.cc) run as a child
process, its outputs checked against the committed golden fixtures (tests/golden/oracle_golden.npz:
the oracle's keypoints / descriptors of synth_image(2) and ComputeStereoMatches of synth_stereo(5))
and, where no fixture covers a result, the oracle on the same inputs (the right image's extraction,
SearchByProjection over the map points the consumer generated and reports back).
The CPU tests check that the consumer links against the library by name and fails loudly without a
HIP device."""
import hashlib
import os
import struct
import subprocess

import numpy as np
import pytest

from orb_slam3_ros_amd import build as B
from orb_slam3_ros_amd.extractor import KEYPOINT_DTYPE
from orb_slam3_ros_amd.matcher import MAP_POINT_DTYPE, MatchFrame
from orb_slam3_ros_amd.synth import synth_image, synth_stereo

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.npz")


@pytest.fixture(scope="module")
def consumer(orbfe_lib):
    return B.build_capi_consumer()


def _run(binary, tmp_path, left, right, nf, n_mps, th, bf, fx):
    h, w = left.shape
    job = tmp_path / "job.bin"
    out = tmp_path / "out.bin"
    job.write_bytes(struct.pack("<5i2f", w, h, nf, n_mps, int(round(th * 100)), bf, fx) +
                    np.ascontiguousarray(left).tobytes() + np.ascontiguousarray(right).tobytes())
    r = subprocess.run([binary, str(job), str(out)], capture_output=True, text=True, timeout=120)
    return r, out


def _parse(buf, n_mps):
    o = 0

    def take(dtype, count):
        nonlocal o
        a = np.frombuffer(buf, dtype, count, o)
        o += a.nbytes
        return a

    sides = []
    for _ in range(2):
        mono, n = take("<i4", 2)
        kp = take(KEYPOINT_DTYPE, n)
        desc = take(np.uint8, n * 32).reshape(n, 32)
        sides.append((int(mono), kp, desc))
    levels = int(take("<i4", 1)[0])
    scale = take("<f4", levels)
    nl = len(sides[0][1])
    nmatch = int(take("<i4", 1)[0])
    ur = take("<f4", nl)
    dp = take("<f4", nl)
    mps = take(MAP_POINT_DTYPE, n_mps)
    nsbp = int(take("<i4", 1)[0])
    mvp = take("<i4", nl)
    assert o == len(buf)
    return sides, scale, nmatch, ur, dp, mps, nsbp, mvp


def _check_sbp(oracle_lib, sides, scale, ur, mps, nsbp, mvp, w, h, bf, th):
    F = MatchFrame(sides[0][1], sides[0][2], (0.0, w, 0.0, h), scale, uright=ur, mbf=bf)
    mvp_o = np.full(len(sides[0][1]), -1, np.int32)
    obs = np.zeros(len(mvp_o), np.int32)
    no = oracle_lib.OracleMatcher(0.8).sbp_local(F, mvp_o, obs, np.ascontiguousarray(mps), th)
    assert nsbp == no > 0
    np.testing.assert_array_equal(mvp, mvp_o)


def test_consumer_links_by_name(consumer):
    r = subprocess.run(["readelf", "-d", consumer], capture_output=True, text=True, check=True)
    assert "[liborbfe.so]" in r.stdout and "$ORIGIN/../../orb_slam3_ros_amd" in r.stdout


def test_consumer_fails_loudly_without_device(consumer, tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is visible")
    img = np.zeros((48, 64), np.uint8)
    r, _ = _run(consumer, tmp_path, img, img, 500, 10, 3.0, 48.0, 435.2)
    assert r.returncode == 1 and "create failed" in r.stderr


@pytest.mark.gpu
def test_consumer_stereo_golden(consumer, oracle_lib, tmp_path):
    """Frame(stereo) + SearchByProjection through the consumer on the golden stereo pair."""
    g = np.load(GOLDEN)
    left, right = synth_stereo(5)
    assert hashlib.sha256(left.tobytes() + right.tobytes()).digest() == g["stereo_img_sha"].tobytes()
    bf, fx, th, n_mps = 0.110078 * 435.2, 435.2, 3.0, 4000
    r, out = _run(consumer, tmp_path, left, right, 1200, n_mps, th, bf, fx)
    assert r.returncode == 0, r.stderr
    sides, scale, nmatch, ur, dp, mps, nsbp, mvp = _parse(out.read_bytes(), n_mps)
    assert nmatch == int(g["stereo_nmatch"][0])
    np.testing.assert_array_equal(ur.view(np.uint32), g["stereo_uright"].view(np.uint32))
    np.testing.assert_array_equal(dp.view(np.uint32), g["stereo_depth"].view(np.uint32))
    for side, img in ((0, left), (1, right)):
        mono, okp, odesc = oracle_lib.OracleExtractor(1200, 1.2, 8, 20, 7)(img)
        assert sides[side][0] == mono
        np.testing.assert_array_equal(sides[side][1].view(np.uint8), okp.view(np.uint8))
        np.testing.assert_array_equal(sides[side][2], odesc)
    _check_sbp(oracle_lib, sides, scale, ur, mps, nsbp, mvp, 752, 480, bf, th)


@pytest.mark.gpu
@pytest.mark.parametrize("th", [1.0, 5.0])
def test_consumer_extract_golden(consumer, oracle_lib, tmp_path, th):
    """ORBextractor::operator() through the consumer on the euroc_stereo_l fixture image (both
    extractors see it, so both sides must equal the fixture)."""
    g = np.load(GOLDEN)
    w, h, nf, _, _ = (int(v) for v in g["euroc_stereo_l_meta"])
    img = synth_image(2, w, h)
    assert hashlib.sha256(img.tobytes()).digest() == g["euroc_stereo_l_img_sha"].tobytes()
    r, out = _run(consumer, tmp_path, img, img, nf, 3000, th, 48.0, 435.2)
    assert r.returncode == 0, r.stderr
    sides, scale, nmatch, ur, dp, mps, nsbp, mvp = _parse(out.read_bytes(), 3000)
    for mono, kp, desc in sides:
        assert mono == int(g["euroc_stereo_l_mono"][0])
        np.testing.assert_array_equal(kp.view(np.uint8).reshape(-1, 28), g["euroc_stereo_l_kp"])
        np.testing.assert_array_equal(desc, g["euroc_stereo_l_desc"])
    _check_sbp(oracle_lib, sides, scale, ur, mps, nsbp, mvp, w, h, 48.0, th)
