"""CPU: liborbfe.so builds for gfx950, loads, and exports every function include/orbfe.h declares
(no compute calls: there is no GPU here)."""
import ctypes
import os
import re

HDR = os.path.join(os.path.dirname(os.path.dirname(__file__)), "include", "orbfe.h")


def _declared_functions():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(orbfe_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    fns = _declared_functions()
    for required in ("orbfe_extractor_create", "orbfe_extract", "orbfe_extract_batch", "orbfe_pyramid_level",
                     "orbfe_stereo_match", "orbfe_stereo_match_batch", "orbfe_descriptor_distance"):
        assert required in fns


def test_library_exports_every_declared_symbol(orbfe_lib):
    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(__file__)), "orb_slam3_ros_amd", "liborbfe.so"))
    missing = [f for f in _declared_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_descriptor_distance_host_entry(orbfe_lib):
    import numpy as np
    a = np.zeros(32, np.uint8)
    b = np.zeros(32, np.uint8)
    b[0], b[31] = 0xFF, 0x01
    assert orbfe_lib.orbfe_descriptor_distance(a.ctypes.data, b.ctypes.data) == 9


def test_triangulation_epi_capacity_is_reported():
    """ORBFE_E_CAPACITY of orbfe_search_for_triangulation_epi (> 16 M candidate slots: one shared
    vocabulary node of 4100 x 4100 entries) reaches a Python caller as OrbfeCapacityError, before any
    device work (this runs without a GPU), so the caller can keep its CPU body."""
    import numpy as np
    import pytest
    from orb_slam3_ros_amd import synth_match as sm
    from orb_slam3_ros_amd._lib import OrbfeCapacityError
    from orb_slam3_ros_amd.matcher import FeatureVector, ORBmatcher
    rng = np.random.default_rng(3)
    n = 4100
    A, B = sm.synth_frame(rng, n, stereo=False), sm.synth_frame(rng, n, stereo=False)
    fv = FeatureVector({7: list(range(n))})
    mp = np.full(n, -1, np.int32)
    calls = []
    with pytest.raises(OrbfeCapacityError):
        ORBmatcher(0.6, True).SearchForTriangulationEpi(A, mp, fv, B, mp.copy(), fv, np.zeros(2, np.float32),
                                                        lambda i, j: calls.append((i, j)) or True)
    assert not calls
