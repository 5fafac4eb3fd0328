"""GPU parity of the BATCHED product path — the path bench.py times.

orbfe_extract_batch over an interleaved [2F, H, W] device tensor of left/right images plus the
same-handle stride-2 orbfe_stereo_match_batch (h, 0, 2, h, 1, 2, F) (or the batched fisheye kNN),
driven through orb_slam3_ros_amd.frontend.StereoFrontEnd exactly as bench.py drives it. This is
the batched form of Frame::Frame (stereo) (Frame.cc:101-197: two ORBextractor::operator() calls,
:122-125, then ComputeStereoMatches, :141 / :811-981) and of the KannalaBrandt8 constructor
(Frame.cc:1007-1075 + ComputeStereoFishEyeMatches' descriptor stage, :1126-1151).

Every frame's keypoints (all 28 bytes), descriptors, monoIndex, uRight / depth bits and nmatch
are compared with the CPU oracle, which runs once per unique synthetic pair; frames map to pairs
through a seeded shuffle so a per-image indexing error cannot alias onto an identical frame.
"""
import concurrent.futures as cf

import numpy as np
import pytest

from orb_slam3_ros_amd.synth import synth_stereo

pytestmark = pytest.mark.gpu

EUROC_BF, EUROC_FX = 0.110078 * 458.654, 458.654
KITTI_BF, KITTI_FX = 0.5327 * 721.5377, 721.5377


def _oracle_pair(oracle_lib, left, right, nfeat, lap_l, lap_r, bf, fx, stereo):
    ol = oracle_lib.OracleExtractor(nfeat, 1.2, 8, 20, 7)
    orr = oracle_lib.OracleExtractor(nfeat, 1.2, 8, 20, 7)
    ml, kl, dl = ol(left, lap_l)
    mr, kr, dr = orr(right, lap_r)
    ref = {"L": (ml, kl, dl), "R": (mr, kr, dr)}
    if stereo == "rectified":
        ur, dp, nm = oracle_lib.stereo_match(ol, orr, kl, dl, kr, dr, bf, fx)
        ref["stereo"] = (ur, dp, nm)
    elif stereo == "fisheye":
        # knnMatch over the lapping rows [monoIndex, n) of each side (Frame.cc:1129-1133)
        good, t, d = oracle_lib.stereo_knn_ratio(dl[ml:], dr[mr:], 0.7)
        l2r = np.full(len(kl), -1, np.int32)
        dist = np.full(len(kl), -1, np.int32)
        sel = t >= 0
        l2r[ml:][sel] = t[sel] + mr
        dist[ml:][sel] = d[sel]
        ref["knn"] = (l2r, dist, good)
    ol.close()
    orr.close()
    return ref


def _oracle_refs(oracle_lib, pairs, nfeat, lap_l, lap_r, bf, fx, stereo):
    with cf.ThreadPoolExecutor(8) as ex:   # ctypes releases the GIL; one oracle instance per task
        futs = [ex.submit(_oracle_pair, oracle_lib, l, r, nfeat, lap_l, lap_r, bf, fx, stereo) for l, r in pairs]
        return [f.result() for f in futs]


def _images(pairs, frame_pair, device):
    import torch
    H, W = pairs[0][0].shape
    host = np.empty((2 * len(frame_pair), H, W), np.uint8)
    for f, p in enumerate(frame_pair):
        host[2 * f], host[2 * f + 1] = pairs[p]
    return torch.from_numpy(host).to(device)


def _check_image(fe, i, ref, what):
    mono, kp, d = fe.host_image(i)
    omono, okp, od = ref
    assert mono == omono, f"{what}: monoIndex {mono} vs {omono}"
    assert len(kp) == len(okp), f"{what}: {len(kp)} keypoints vs {len(okp)}"
    bad = np.nonzero((kp.view(np.uint32).reshape(-1, 7) != okp.view(np.uint32).reshape(-1, 7)).any(1))[0]
    assert bad.size == 0, f"{what}: {bad.size} keypoint records differ, first {bad[:5].tolist()}"
    rows = np.nonzero((d != od).any(1))[0]
    assert rows.size == 0, f"{what}: {rows.size} descriptor rows differ, first {rows[:5].tolist()}"


def _check_batch(fe, frame_pair, refs):
    counts = fe.counts.cpu().numpy()
    nmatch = fe.nmatch.cpu().numpy()
    for f, p in enumerate(frame_pair):
        ref = refs[p]
        _check_image(fe, 2 * f, ref["L"], f"frame {f} left (pair {p})")
        _check_image(fe, 2 * f + 1, ref["R"], f"frame {f} right (pair {p})")
        n = int(counts[2 * f, 0])
        if "stereo" in ref:
            ur, dp, nm = ref["stereo"]
            gur = fe.uright[f, :n].cpu().numpy()
            gdp = fe.depth[f, :n].cpu().numpy()
            assert int(nmatch[f]) == nm, f"frame {f}: nmatch {int(nmatch[f])} vs {nm}"
            assert np.array_equal(gur.view(np.uint32), ur.view(np.uint32)), f"frame {f}: uRight differs"
            assert np.array_equal(gdp.view(np.uint32), dp.view(np.uint32)), f"frame {f}: depth differs"
        if "knn" in ref:
            l2r, dist, good = ref["knn"]
            assert int(nmatch[f]) == good, f"frame {f}: knn ratio passes {int(nmatch[f])} vs {good}"
            assert np.array_equal(fe.l2r[f, :n].cpu().numpy(), l2r), f"frame {f}: left->right candidates differ"
            assert np.array_equal(fe.l2r_dist[f, :n].cpu().numpy(), dist), f"frame {f}: distances differ"
            assert (fe.l2r[f, n:].cpu().numpy() == -1).all()


def _frame_map(nframes, nunique, seed):
    rng = np.random.default_rng(seed)
    m = np.concatenate([np.arange(nunique), rng.integers(0, nunique, nframes - nunique)])
    return rng.permutation(m)[:nframes]


def test_bench_path_config2_f512(gpu, oracle_lib):
    """BASELINE config 2 at bench.py's batch: 512 stereo frames = 1024 images per launch (k_resize_s
    chain with k_fast overlapped on a side stream, octree, describe, stereo)."""
    from orb_slam3_ros_amd.frontend import StereoFrontEnd
    F, U = 512, 32
    pairs = [synth_stereo(500 + i, 752, 480) for i in range(U)]
    fmap = _frame_map(F, U, 1)
    refs = _oracle_refs(oracle_lib, pairs, 1000, (0, 0), (0, 0), EUROC_BF, EUROC_FX, "rectified")
    images = _images(pairs, fmap, gpu)
    fe = StereoFrontEnd(F, 752, 480, nfeatures=1000, bf=EUROC_BF, fx=EUROC_FX, device=gpu)
    for _ in range(2):   # a repeated run over the same buffers must give the same answer
        fe.run(images)
        _check_batch(fe, fmap, refs)
    fe.close()


def test_bench_path_pipelines_bound_slab(gpu, oracle_lib):
    """pipelines=2 (two handles / streams, sub-batch offsets) with the outputs bound to the views
    of one flat slab, as the multi-GPU bench binds distributed.SlabExchange buffers."""
    import torch
    from orb_slam3_ros_amd import distributed as odist
    from orb_slam3_ros_amd.frontend import StereoFrontEnd
    F, U = 37, 9   # odd: the two pipelines get 18 and 19 frames
    pairs = [synth_stereo(600 + i, 752, 480) for i in range(U)]
    fmap = _frame_map(F, U, 2)
    refs = _oracle_refs(oracle_lib, pairs, 1000, (0, 0), (0, 0), EUROC_BF, EUROC_FX, "rectified")
    images = _images(pairs, fmap, gpu)
    fe = StereoFrontEnd(F, 752, 480, nfeatures=1000, bf=EUROC_BF, fx=EUROC_FX, device=gpu, pipelines=2)
    slab = torch.zeros(odist.slab_bytes(2 * F, fe.cap), dtype=torch.uint8, device=gpu)
    fe.bind_outputs(*odist.slab_views(slab, 2 * F, fe.cap))
    fe.run(images)
    torch.cuda.synchronize()
    _check_batch(fe, fmap, refs)
    # the slab bytes are the slot records the all-gather moves
    counts, kps, desc = odist.slab_views(slab, 2 * F, fe.cap)
    assert torch.equal(counts, fe.counts) and torch.equal(desc, fe.desc)
    fe.close()


def test_config3_kitti_batch(gpu, oracle_lib):
    """BASELINE config 3: 1241x376, nFeatures 2000, ComputeStereoMatches at KITTI's baseline."""
    from orb_slam3_ros_amd.frontend import StereoFrontEnd
    F, U = 16, 6
    pairs = [synth_stereo(700 + i, 1241, 376) for i in range(U)]
    fmap = _frame_map(F, U, 3)
    refs = _oracle_refs(oracle_lib, pairs, 2000, (0, 0), (0, 0), KITTI_BF, KITTI_FX, "rectified")
    images = _images(pairs, fmap, gpu)
    fe = StereoFrontEnd(F, 1241, 376, nfeatures=2000, bf=KITTI_BF, fx=KITTI_FX, device=gpu)
    fe.run(images)
    _check_batch(fe, fmap, refs)
    assert fe.nmatch.cpu().numpy().min() > 100
    fe.close()


@pytest.mark.parametrize("laps", [((0, 511), (0, 511)), ((0, 400), (100, 511))])
def test_config4_fisheye_batch(gpu, oracle_lib, laps):
    """BASELINE config 4 per-GPU step: 512x512 KannalaBrandt8 stereo, each side with its camera's
    vLappingArea, plus the batched knnMatch(k=2) + ratio over the lapping rows."""
    from orb_slam3_ros_amd.frontend import StereoFrontEnd
    F, U = 8, 4
    pairs = [synth_stereo(800 + i, 512, 512) for i in range(U)]
    fmap = _frame_map(F, U, 4)
    refs = _oracle_refs(oracle_lib, pairs, 1000, laps[0], laps[1], 0.0, 1.0, "fisheye")
    images = _images(pairs, fmap, gpu)
    fe = StereoFrontEnd(F, 512, 512, nfeatures=1000, device=gpu, lap_left=laps[0], lap_right=laps[1],
                        stereo="fisheye")
    fe.run(images)
    _check_batch(fe, fmap, refs)
    assert fe.nmatch.cpu().numpy().min() > 0
    fe.close()


def test_rejected_size_keeps_handle(gpu, oracle_lib):
    """A size the geometry rejects (a level below the FAST grid minimum) leaves the handle intact:
    good size -> rejected size (ORBFE_E_ARG) -> good size again, bit-exact."""
    from orb_slam3_ros_amd import _lib
    from orb_slam3_ros_amd.extractor import ORBextractor
    img = synth_stereo(901, 752, 480)[0]
    ora = oracle_lib.OracleExtractor(1000, 1.2, 8, 20, 7)
    omono, okp, od = ora(img)
    ext = ORBextractor(1000, 1.2, 8, 20, 7)
    for _ in range(2):
        mono, kp, d = ext(img)
        assert mono == omono and np.array_equal(kp.view(np.uint32), okp.view(np.uint32)) and np.array_equal(d, od)
        with pytest.raises(_lib.OrbfeError):
            ext(np.zeros((150, 200), np.uint8) + 7)
    ext.close()


def test_bound_outputs_capacity(gpu):
    """Outputs bound for fewer images than the batch: ORBFE_E_CAPACITY, never a silent write
    into the handle's own buffers."""
    import ctypes
    import torch
    from orb_slam3_ros_amd import _lib
    lib = _lib.load()
    h = ctypes.c_void_p()
    _lib.check(lib.orbfe_extractor_create(1000, 1.2, 8, 20, 7, ctypes.byref(h)), "create")
    cap = lib.orbfe_extractor_capacity(h, 752, 480)
    kps = torch.zeros((2, cap, 7), dtype=torch.int32, device=gpu)
    desc = torch.zeros((2, cap, 32), dtype=torch.uint8, device=gpu)
    cnt = torch.zeros((2, 2), dtype=torch.int32, device=gpu)
    lib.orbfe_set_batch_outputs(h, kps.data_ptr(), desc.data_ptr(), cnt.data_ptr(), 2)
    imgs = torch.zeros((3, 480, 752), dtype=torch.uint8, device=gpu)
    ptrs = (ctypes.c_void_p * 3)(*[imgs[i].data_ptr() for i in range(3)])
    assert lib.orbfe_extract_batch(h, 3, ptrs, 752, 480, 752, 0, 0, None) == _lib.ORBFE_E_CAPACITY
    assert lib.orbfe_extract_batch(h, 2, ptrs, 752, 480, 752, 0, 0, None) == 0
    torch.cuda.synchronize()
    lib.orbfe_extractor_destroy(h)
