"""ctypes binding of liborbfe.so (the C-ABI declared in include/orbfe.h).

The library is built in-tree by orb_slam3_ros_amd.build.build_library() (hipcc, gfx950). There is
no CPU fallback: if the shared object is missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liborbfe.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "orbfe.h")

ORBFE_OK = 0
ORBFE_E_EMPTY = -1
ORBFE_E_ARG = -2
ORBFE_E_DEVICE = -3
ORBFE_E_CAPACITY = -4
ORBFE_NUM_STAGES = 3
STAGE_NAMES = ("pyramid_fast", "octree", "describe")


# orbfe_epipolar_fn: int32_t (*)(void* ctx, int32_t idx1, int32_t idx2)
EPIPOLAR_FN = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32)


class OrbKeyPoint(ctypes.Structure):
    """cv::KeyPoint byte layout (28 B)."""
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("size", ctypes.c_float),
                ("angle", ctypes.c_float), ("response", ctypes.c_float),
                ("octave", ctypes.c_int32), ("class_id", ctypes.c_int32)]


_c_int, _c_float, _vp = ctypes.c_int, ctypes.c_float, ctypes.c_void_p
_P_int, _P_float = ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_float)

_SIGS = {
    "orbfe_extractor_create": (_c_int, [_c_int, _c_float, _c_int, _c_int, _c_int, ctypes.POINTER(_vp)]),
    "orbfe_extractor_destroy": (None, [_vp]),
    "orbfe_extractor_levels": (_c_int, [_vp]),
    "orbfe_extractor_scale_info": (_c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "orbfe_extractor_capacity": (_c_int, [_vp, _c_int, _c_int]),
    "orbfe_extract": (_c_int, [_vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _c_int, _P_int]),
    "orbfe_pyramid_level": (_c_int, [_vp, _c_int, _c_int, _vp, _c_int, _P_int, _P_int]),
    "orbfe_extract_batch": (_c_int, [_vp, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _vp]),
    "orbfe_extract_batch_laps": (_c_int, [_vp, _c_int, _vp, _c_int, _c_int, _c_int, _vp, _vp]),
    "orbfe_batch_outputs": (_c_int, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_vp), _P_int]),
    "orbfe_set_stage_timing": (_c_int, [_vp, _c_int]),
    "orbfe_extractor_set_opencv_model": (_c_int, [_vp, _c_int, _c_int]),
    "orbfe_extractor_get_opencv_model": (_c_int, [_vp, _P_int, _P_int]),
    "orbfe_set_batch_outputs": (_c_int, [_vp, _vp, _vp, _vp, _c_int]),
    "orbfe_get_stage_timing": (_c_int, [_vp, _vp]),
    "orbfe_get_call_timing": (_c_int, [_vp, _vp]),
    "orbfe_stereo_match_batch": (_c_int, [_vp, _c_int, _c_int, _vp, _c_int, _c_int, _c_int, _c_float, _c_float,
                                          _vp, _vp, _vp, _vp]),
    "orbfe_stereo_match": (_c_int, [_vp, _vp, _c_float, _c_float, _vp, _vp]),
    "orbfe_frame_stereo": (_c_int, [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_float, _c_float,
                                    _vp, _vp, _c_int, _P_int, _P_int, _vp, _vp, _c_int, _P_int, _P_int, _vp, _vp]),
    "orbfe_frame_fisheye": (_c_int, [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_float,
                                     _vp, _vp, _c_int, _P_int, _P_int, _vp, _vp, _c_int, _P_int, _P_int, _vp, _vp]),
    "orbfe_descriptor_distance": (_c_int, [_vp, _vp]),
    "orbfe_debug_copy": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _c_int]),
    "orbfe_debug_block_sort": (_c_int, [_vp, _c_int]),
    "orbfe_version": (ctypes.c_char_p, []),
    "orbfe_search_by_projection_local": (_c_int, [_vp, _vp, _vp, _vp, _c_int, _c_float, _c_int, _c_float, _c_float]),
    "orbfe_search_by_projection_lastframe": (_c_int, [_vp, _vp, _vp, _vp, _c_int, _c_float, _c_int, _c_int, _c_int]),
    "orbfe_search_by_projection_lastframe_stereo": (_c_int, [_vp, _vp, _vp, _vp, _vp, _c_int, _c_float, _c_int, _c_int,
                                                             _c_int]),
    "orbfe_search_by_projection_lastframe_pose": (_c_int, [_vp, _vp, _vp, _vp, _c_int, _vp, _vp, _vp, _c_float, _c_int,
                                                           _c_int, _c_int]),
    "orbfe_search_by_projection_kf": (_c_int, [_vp, _vp, _vp, _c_int, _c_float, _c_int, _c_int]),
    "orbfe_search_for_initialization": (_c_int, [_vp, _vp, _vp, _vp, _c_int, _c_float, _c_int]),
    "orbfe_search_by_bow": (_c_int, [_vp, _vp, _vp, _c_int, _vp, _vp, _vp, _vp, _c_float, _c_int]),
    "orbfe_copy_stream": (_c_int, [_vp, _vp, ctypes.c_size_t, _vp]),
    "orbfe_search_by_projection_local_device": (_c_int, [_vp, _vp, _vp, _vp, _c_int, _c_float, _c_int, _c_float,
                                                         _c_float, _vp]),
    "orbfe_search_local_points_device": (_c_int, [_vp, _vp, _vp, _c_int, _vp, _vp, _c_float, _c_int, _c_float,
                                                  _c_float, _vp, _vp]),
    "orbfe_search_by_bow_kf": (_c_int, [_vp, _vp, _vp, _c_int, _vp, _vp, _vp, _vp, _c_int, _vp, _vp, _c_float,
                                        _c_int]),
    "orbfe_distinctive_descriptors": (_c_int, [_vp, _vp, _c_int, _vp]),
    "orbfe_search_for_triangulation": (_c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_int, _c_int, _c_int,
                                                _vp]),
    "orbfe_fuse": (_c_int, [_vp, _vp, _vp, _vp, _c_int, _c_float, _c_int, _vp, _vp]),
    "orbfe_search_by_projection_sim3": (_c_int, [_vp, _vp, _vp, _c_int, _vp, _c_int, _c_float, _vp, _vp]),
    "orbfe_search_by_projection_sim3_rig": (_c_int, [_vp, _vp, _vp, _vp, _c_int, _vp, _c_int, _c_float, _vp, _vp]),
    "orbfe_search_for_triangulation_epi": (_c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_int, _c_int, EPIPOLAR_FN,
                                                    _vp, _vp]),
    "orbfe_search_by_sim3": (_c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_float, _vp, _vp]),
    "orbfe_stereo_knn_ratio": (_c_int, [_vp, _c_int, _vp, _c_int, _c_float, _vp, _vp]),
    "orbfe_stereo_knn_slabs": (_c_int, [_vp, _vp, _c_int, _c_int, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_float,
                                        _vp, _vp, _vp, _vp]),
    "orbfe_stereo_knn_batch": (_c_int, [_vp, _c_int, _c_int, _vp, _c_int, _c_int, _c_int, _c_float, _vp, _vp, _vp,
                                        _vp]),
    "orbfe_matcher_set_timing": (_c_int, [_c_int]),
    "orbfe_matcher_set_stats": (_c_int, [_c_int]),
    "orbfe_matcher_last_stats": (_c_int, [_vp]),
    "orbfe_undistort_points": (_c_int, [_vp, _c_int, _vp, _vp, _c_int, _vp]),
    "orbfe_remap_linear": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp, _c_int, _c_int, _vp, _c_int]),
    "orbfe_remap_linear_batch": (_c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp, _c_int, _c_int, _vp, _c_int, _c_int, _vp]),
    "orbfe_vocabulary_load_bin": (_c_int, [_vp, ctypes.c_size_t, ctypes.POINTER(_vp)]),
    "orbfe_vocabulary_create": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, ctypes.POINTER(_vp)]),
    "orbfe_vocabulary_destroy": (None, [_vp]),
    "orbfe_vocabulary_info": (_c_int, [_vp, _vp, _vp, _vp, _vp]),
    "orbfe_vocabulary_transform": (_c_int, [_vp, _vp, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "orbfe_is_in_frustum": (_c_int, [_vp, _vp, _vp, _c_int, _vp]),
    "orbfe_search_local_points": (_c_int, [_vp, _vp, _vp, _c_int, _vp, _vp, _c_float, _c_int, _c_float, _c_float, _vp]),
    "orbfe_matcher_last_ms": (_c_float, []),
    "orbfe_is_in_frustum_rig": (_c_int, [_vp, _vp, _vp, _vp, _c_int, _vp]),
    "orbfe_search_by_bow_kf2": (_c_int, [_vp, _vp, _vp, _c_int, _c_int, _vp, _vp, _vp, _vp, _c_int, _c_int, _vp, _vp,
                                         _c_float, _c_int]),
    "orbfe_fuse_rig": (_c_int, [_vp, _vp, _vp, _vp, _vp, _c_int, _c_float, _c_int, _c_int, _vp, _vp]),
    "orbfe_search_local_points_rig": (_c_int, [_vp, _vp, _vp, _vp, _c_int, _vp, _vp, _c_float, _c_int, _c_float,
                                               _c_float, _vp]),
    "orbfe_search_local_points_rig_device": (_c_int, [_vp, _vp, _vp, _vp, _c_int, _vp, _vp, _c_float, _c_int,
                                                      _c_float, _c_float, _vp, _vp]),
    "orbfe_search_local_points_track": (_c_int, [_vp, _vp, _vp, _vp, _c_int, _vp, _vp, _c_float, _c_int, _c_float,
                                                 _c_float, _vp, _vp]),
    "orbfe_extractor_frame_id": (ctypes.c_uint64, [_vp]),
    "orbfe_frame_device_view": (_c_int, [_vp, ctypes.c_uint64, _vp]),
}

_lib = None


class OrbfeError(RuntimeError):
    pass


class OrbfeCapacityError(OrbfeError):
    """ORBFE_E_CAPACITY: the call's inputs exceed a documented device limit (include/orbfe.h). No
    device work ran and no output was written; the caller keeps its CPU body for this call, as the
    C++ shim does (shim/ORBmatcher_backend_orbfe.cc). The library never falls back by itself."""


def load(path: str | None = None) -> ctypes.CDLL:
    """Load liborbfe.so (raises OrbfeError if it is missing: there is no fallback path)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # ORBFE_LIB: an alternative build of the same library (kernel A/B experiments, tools/)
    p = path or os.environ.get("ORBFE_LIB") or LIB_PATH
    # One HIP runtime per process: torch ships its own libamdhip64.so with the same soname as
    # /opt/rocm's. Import torch first (when present) so liborbfe.so binds to that runtime too;
    # loading ours first would put two runtimes in the process and break device calls.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(p):
        raise OrbfeError(f"liborbfe.so not found at {p}; build it with orb_slam3_ros_amd.build.build_library()")
    lib = ctypes.CDLL(p)
    for name, (res, args) in _SIGS.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            # an older build (a kernel A/B baseline) may predate an entry point, but only when that
            # is asked for explicitly (ORBFE_LIB_PARTIAL=1); the product library, reached by any
            # path, must export every symbol (tests/test_capi.py)
            if os.environ.get("ORBFE_LIB_PARTIAL") != "1" or os.path.realpath(p) == os.path.realpath(LIB_PATH):
                raise
            continue
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(rc: int, what: str) -> int:
    if rc < 0 and rc != ORBFE_E_EMPTY:
        names = {ORBFE_E_ARG: "bad argument", ORBFE_E_DEVICE: "HIP device error", ORBFE_E_CAPACITY: "capacity"}
        cls = OrbfeCapacityError if rc == ORBFE_E_CAPACITY else OrbfeError
        raise cls(f"{what} failed: {names.get(rc, rc)}")
    return rc
