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
from orb_slam3_ros_amd.matcher import FeatureVector, ORBmatcher, compute_distinctive_descriptors

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
