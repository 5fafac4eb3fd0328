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


@pytest.fixture(scope="module")
def seq_job(tmp_path_factory):
    import bench
    p = tmp_path_factory.mktemp("seq") / "seq.bin"
    return str(bench.write_sequence_job(str(p), 24, nf=1000, window=20))


@pytest.fixture(scope="module")
def tracking_cpu_bin(oracle_lib):
    return B.build_tracking_cpu()


def _tracking_records(buf, two_cams=False):
    """Per frame {n_left, n_right, n_stereo, sbp_th, sbp_matches, n_to_match, local_matches, mvp[n_left]}
    (two-camera frames: mvp[n_left + n_right], both cameras' slots)."""
    a = np.frombuffer(buf, "<i4")
    out, o = [], 0
    while o < len(a):
        rec = a[o:o + 7]
        n = rec[0] + (rec[1] if two_cams else 0)
        mvp = a[o + 7:o + 7 + n]
        out.append((rec.copy(), mvp.copy()))
        o += 7 + n
    return out


@pytest.fixture(scope="module")
def seq_job_kb8(tmp_path_factory):
    import bench
    p = tmp_path_factory.mktemp("seqkb8") / "seq.bin"
    return str(bench.write_sequence_job(str(p), 24, 512, 512, 1000, 20, 31, (256.0, 256.0)))


def test_tracking_kb8_cpu_sequence(tracking_cpu_bin, seq_job_kb8, tmp_path):
    """The KannalaBrandt8 two-camera Tracking loop on the CPU restatement (tests/native/tracking_kb8.h):
    deterministic, and every call does real work (ratio-test stereo pairs, a last-frame search over
    both cameras' slots, a local map projected into both cameras)."""
    import json
    outs = []
    for i in range(2):
        o = tmp_path / f"k{i}.out"
        r = subprocess.run([tracking_cpu_bin, "--kb8", "10", seq_job_kb8, str(o)], capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr
        outs.append(o.read_bytes())
    assert outs[0] == outs[1]
    recs = _tracking_records(outs[0], two_cams=True)
    assert len(recs) == 10
    st = json.loads(r.stdout.strip().splitlines()[-1])
    assert st["mean"]["stereo_matches"] > 200 and st["mean"]["last_frame_matches"] > 0.5 * st["mean"]["last_frame_points"]
    assert st["mean"]["local_to_match"] > 50 and st["mean"]["local_matches"] > 10
    assert any((mvp[rec[0]:] >= 0).any() for rec, mvp in recs[1:])   # right-camera slots matched too


@pytest.mark.gpu
def test_tracking_kb8_sequence_matches_cpu(consumer, tracking_cpu_bin, seq_job_kb8, tmp_path):
    """The two-camera Tracking frame through the C-ABI (both extractions with vLappingArea
    {0, 511} and the kNN in one orbfe_frame_fisheye call, orbfe_search_by_projection_lastframe_pose,
    orbfe_search_local_points_track with a KannalaBrandt8 rig) over 24 frames, against the same loop
    on the CPU restatement: every frame's counts and both cameras' slots identical."""
    g, c = tmp_path / "gpu.out", tmp_path / "cpu.out"
    r = subprocess.run([consumer, "--tracking-kb8", "24", seq_job_kb8, str(g)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    rc = subprocess.run([tracking_cpu_bin, "--kb8", "24", seq_job_kb8, str(c)], capture_output=True, text=True,
                        timeout=600)
    assert rc.returncode == 0, rc.stderr
    gr, cr = _tracking_records(g.read_bytes(), True), _tracking_records(c.read_bytes(), True)
    assert len(gr) == len(cr) == 24
    for k, ((ga, gm), (ca, cm)) in enumerate(zip(gr, cr)):
        np.testing.assert_array_equal(ga, ca, err_msg=f"frame {k} counts")
        np.testing.assert_array_equal(gm, cm, err_msg=f"frame {k} mvpMapPoints")


def test_tracking_cpu_sequence_deterministic(tracking_cpu_bin, seq_job, tmp_path):
    """The CPU Tracking-frame loop (oracle restatement) is deterministic and does real work: the motion
    model finds most last-frame points, SearchLocalPoints projects a growing local map."""
    import json
    outs = []
    for i in range(2):
        o = tmp_path / f"cpu{i}.out"
        r = subprocess.run([tracking_cpu_bin, "12", seq_job, str(o)], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        outs.append(o.read_bytes())
    assert outs[0] == outs[1]
    recs = _tracking_records(outs[0])
    assert len(recs) == 12
    st = json.loads(r.stdout.strip().splitlines()[-1])
    assert st["mean"]["last_frame_matches"] > 0.5 * st["mean"]["last_frame_points"] > 200
    assert st["mean"]["local_to_match"] > 100 and st["mean"]["local_matches"] > 10
    for rec, mvp in recs[1:]:
        assert rec[4] == (mvp >= 0).sum() - rec[6] or rec[4] >= 20


@pytest.mark.gpu
def test_tracking_sequence_matches_cpu(consumer, tracking_cpu_bin, seq_job, tmp_path):
    """A whole Tracking frame through the C-ABI (orbfe_frame_stereo, SearchByProjection(CurrentFrame,
    LastFrame, 7), SearchLocalPoints) over a 24-frame sequence, against the same loop on the CPU
    restatement: every frame's counts and mvpMapPoints identical (the loop feeds each frame's results
    into the next frame's inputs, so one difference would propagate)."""
    g, c = tmp_path / "gpu.out", tmp_path / "cpu.out"
    r = subprocess.run([consumer, "--tracking", "24", seq_job, str(g)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    rc = subprocess.run([tracking_cpu_bin, "24", seq_job, str(c)], capture_output=True, text=True, timeout=600)
    assert rc.returncode == 0, rc.stderr
    gr, cr = _tracking_records(g.read_bytes()), _tracking_records(c.read_bytes())
    assert len(gr) == len(cr) == 24
    for k, ((ga, gm), (ca, cm)) in enumerate(zip(gr, cr)):
        np.testing.assert_array_equal(ga, ca, err_msg=f"frame {k} counts")
        np.testing.assert_array_equal(gm, cm, err_msg=f"frame {k} mvpMapPoints")


@pytest.mark.gpu
def test_latency_mode_sequence(consumer, seq_job):
    """The drop-in latency harness over the sequence: both forms run and report the same work."""
    import json
    r = subprocess.run([consumer, "--latency", "10", seq_job], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["distinct_pairs"] == 24 and d["frames"] == 10
    assert d["frame_call"]["keypoints_lr"] > 1800 and d["frame_call"]["stereo_matches"] > 300
    assert d["frame_call"]["frame_ms"] > 0 and d["threads"]["frame_ms"] > 0
