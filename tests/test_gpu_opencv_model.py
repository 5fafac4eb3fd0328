"""GPU parity under every OpenCV-behaviour model the boundary exposes (orbfe_extractor_set_opencv_model).

The reference's cv::resize (ORBextractor.cc:1183) and cv::GaussianBlur (:1133) results depend on
how its OpenCV was built (the universal-intrinsic lane count of the resize vertical
pass, the Q8 blur kernel quantisation). The library and the oracle both carry the two switches;
here each (lanes, blur) setting runs the HIP path and the oracle under the SAME setting and
compares every pyramid level, every keypoint field and every descriptor bit-exactly, at the
BASELINE config 2 and config 3 geometries.
"""
import numpy as np
import pytest

from orb_slam3_ros_amd.synth import synth_image, synth_stereo

pytestmark = pytest.mark.gpu

LANES = [0, 8, 16, 32, 64]
BLURS = [0, 1]
GEOMS = [(752, 480, 1000), (1241, 376, 2000)]


def _check(ext, ora, img, nlevels=8):
    mono_g, kp_g, d_g = ext(img, None, (0, 0))
    mono_o, kp_o, d_o = ora(img)
    for lv in range(nlevels):
        pg, po = ext.pyramid_level(lv), ora.pyramid_level(lv)
        assert pg.shape == po.shape
        bad = np.argwhere(pg != po)
        assert bad.size == 0, f"pyramid level {lv}: {len(bad)} px differ, first {bad[:3].tolist()}"
    assert mono_g == mono_o and len(kp_g) == len(kp_o)
    assert np.array_equal(kp_g.view(np.uint32), kp_o.view(np.uint32)), "keypoint records differ"
    rows = np.nonzero((d_g != d_o).any(axis=1))[0]
    assert rows.size == 0, f"{rows.size} descriptor rows differ, first {rows[:5].tolist()}"
    return len(kp_g)


@pytest.mark.parametrize("blur", BLURS)
@pytest.mark.parametrize("lanes", LANES)
@pytest.mark.parametrize("w,h,nfeat", GEOMS)
def test_opencv_model_matches_oracle(w, h, nfeat, lanes, blur, gpu, oracle_lib):
    from orb_slam3_ros_amd.extractor import ORBextractor
    img = synth_image(300 + w + lanes, w, h)
    ext = ORBextractor(nfeat, 1.2, 8, 20, 7)
    ext.set_opencv_model(lanes, blur)
    assert ext.opencv_model() == (lanes, blur)
    ora = oracle_lib.OracleExtractor(nfeat, 1.2, 8, 20, 7, resize_simd_lanes=lanes, blur_variant=blur)
    assert _check(ext, ora, img) >= 0.9 * nfeat
    ext.close()


def test_models_differ_where_expected(gpu, oracle_lib):
    """The switches are live: a scalar resize changes some pyramid pixel and the other blur kernel
    some descriptor bit (so the parametrised test above compares distinct outputs)."""
    from orb_slam3_ros_amd.extractor import ORBextractor
    img = synth_image(77, 752, 480)
    ext = ORBextractor(1000, 1.2, 8, 20, 7)
    _, _, d16 = ext(img)
    p16 = [ext.pyramid_level(lv) for lv in range(1, 8)]
    ext.set_opencv_model(0, 0)
    ext(img)
    p0 = [ext.pyramid_level(lv) for lv in range(1, 8)]
    assert any((a != b).any() for a, b in zip(p16, p0)), "lanes 0 vs 16: identical pyramids"
    ext.set_opencv_model(16, 1)
    _, _, d_round = ext(img)
    assert [np.array_equal(a, b) for a, b in zip(p16, [ext.pyramid_level(lv) for lv in range(1, 8)])] == [True] * 7
    assert d_round.shape != d16.shape or (d_round != d16).any(), "blur 0 vs 1: identical descriptors"
    ext.close()


def test_model_switch_on_live_handle(gpu, oracle_lib):
    """Switching back and forth on one handle (buffers rebuilt each time) stays bit-exact."""
    from orb_slam3_ros_amd.extractor import ORBextractor
    img = synth_image(78, 752, 480)
    ext = ORBextractor(1000, 1.2, 8, 20, 7)
    for lanes, blur in [(32, 1), (16, 0), (0, 1), (16, 0)]:
        ext.set_opencv_model(lanes, blur)
        ora = oracle_lib.OracleExtractor(1000, 1.2, 8, 20, 7, resize_simd_lanes=lanes, blur_variant=blur)
        _check(ext, ora, img)
    ext.close()


@pytest.mark.parametrize("lanes,blur", [(7, 0), (16, 2), (-1, 0), (128, 1)])
def test_model_rejects_bad_values(lanes, blur, gpu):
    from orb_slam3_ros_amd import _lib
    from orb_slam3_ros_amd.extractor import ORBextractor
    ext = ORBextractor(1000, 1.2, 8, 20, 7)
    with pytest.raises(_lib.OrbfeError):
        ext.set_opencv_model(lanes, blur)
    assert ext.opencv_model() == (16, 0)
    ext.close()


@pytest.mark.parametrize("lanes,blur", [(32, 1), (0, 0)])
def test_batched_stereo_under_model(lanes, blur, gpu, oracle_lib):
    """The batched front end (bench path) under a non-default model: keypoints, descriptors and
    ComputeStereoMatches of every frame against the oracle with the same model."""
    import torch
    from orb_slam3_ros_amd.frontend import StereoFrontEnd
    W, H, F = 752, 480, 8
    bf, fx = 0.110078 * 458.654, 458.654
    pairs = [synth_stereo(900 + i, W, H) for i in range(F)]
    host = np.stack([im for p in pairs for im in p])
    dev = torch.device("cuda", 0)
    images = torch.from_numpy(host).to(dev)
    fe = StereoFrontEnd(F, W, H, bf=bf, fx=fx, device=dev)
    fe.set_opencv_model(lanes, blur)
    fe.run(images)
    torch.cuda.synchronize()
    for f, (left, right) in enumerate(pairs):
        ol = oracle_lib.OracleExtractor(1000, 1.2, 8, 20, 7, resize_simd_lanes=lanes, blur_variant=blur)
        orr = oracle_lib.OracleExtractor(1000, 1.2, 8, 20, 7, resize_simd_lanes=lanes, blur_variant=blur)
        ml, kl, dl = ol(left)
        mr, kr, dr = orr(right)
        for side, (m, k, d) in enumerate(((ml, kl, dl), (mr, kr, dr))):
            gm, gk, gd = fe.host_image(2 * f + side)
            assert gm == m and np.array_equal(gk.view(np.uint32), k.view(np.uint32)) and np.array_equal(gd, d), \
                f"frame {f} side {side}"
        ur, dp, nm = oracle_lib.stereo_match(ol, orr, kl, dl, kr, dr, bf, fx)
        n = len(kl)
        assert int(fe.nmatch[f]) == nm
        assert np.array_equal(fe.uright[f, :n].cpu().numpy().view(np.uint32), ur.view(np.uint32))
        assert np.array_equal(fe.depth[f, :n].cpu().numpy().view(np.uint32), dp.view(np.uint32))
    fe.close()
