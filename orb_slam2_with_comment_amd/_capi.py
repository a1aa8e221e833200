"""ctypes binding of include/orbmi.h (liborbmi.so, built in-tree by build.py).

There is no fallback: if the HIP library is missing or fails to load, importing the
product classes raises.  Only the C-ABI is used; no torch types cross the boundary.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from .build import LIB

ORBMI_OK = 0
ORBMI_E_ARG = -1
ORBMI_E_HIP = -2
ORBMI_E_CAP = -3
ORBMI_E_UNSUPPORTED = -4
ORBMI_E_STATE = -5
STAGES = ["pyr_level0", "pyr_resize", "fast", "octree", "describe", "stereo_rows", "stereo_match",
          "stereo_filter", "blur"]
NUM_STAGES = 16
_NAMES = {ORBMI_E_ARG: "ORBMI_E_ARG", ORBMI_E_HIP: "ORBMI_E_HIP", ORBMI_E_CAP: "ORBMI_E_CAP",
          ORBMI_E_UNSUPPORTED: "ORBMI_E_UNSUPPORTED", ORBMI_E_STATE: "ORBMI_E_STATE"}


class OrbmiError(RuntimeError):
    def __init__(self, func: str, code: int):
        super().__init__(f"{func} returned {_NAMES.get(code, code)}")
        self.code = code


class Keypoint(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("size", C.c_float), ("angle", C.c_float),
                ("response", C.c_float), ("octave", C.c_int32), ("class_id", C.c_int32)]


KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KP_DTYPE.itemsize == C.sizeof(Keypoint) == 28

_vp, _i, _f, _sz = C.c_void_p, C.c_int, C.c_float, C.c_size_t
_PROTOS = {
    "orbmi_extractor_create": (_i, [_i, _i, _f, _i, _i, _i, C.POINTER(_vp)]),
    "orbmi_extractor_destroy": (None, [_vp]),
    "orbmi_extract": (_i, [_vp, _vp, _i, _i, _sz, _vp, _vp, _i, C.POINTER(_i)]),
    "orbmi_extract_batch_device": (_i, [_vp, _vp, _i, _i, _i, _sz, _sz, _vp, _vp, _vp, _i]),
    "orbmi_extract_batch_host": (_i, [_vp, _vp, _i, _i, _i, _sz, _vp, _vp, _vp, _i]),
    "orbmi_extractor_synchronize": (_i, [_vp]),
    "orbmi_extractor_get_levels": (_i, [_vp]),
    "orbmi_extractor_get_scale_factor": (_f, [_vp]),
    "orbmi_extractor_get_scale_factors": (_i, [_vp, _vp]),
    "orbmi_extractor_get_inverse_scale_factors": (_i, [_vp, _vp]),
    "orbmi_extractor_get_scale_sigma_squares": (_i, [_vp, _vp]),
    "orbmi_extractor_get_inverse_scale_sigma_squares": (_i, [_vp, _vp]),
    "orbmi_extractor_get_features_per_level": (_i, [_vp, _vp]),
    "orbmi_extractor_get_pyramid_level": (_i, [_vp, _i, _i, _i, _vp, _sz, C.POINTER(_i), C.POINTER(_i)]),
    "orbmi_compute_stereo_matches": (_i, [_vp, _i, _vp, _i, _f, _f, _vp, _vp, _i]),
    "orbmi_compute_stereo_matches_batch_device": (_i, [_vp, _f, _f, _vp, _vp]),
    "orbmi_matcher_create": (_i, [_i, C.POINTER(_vp)]),
    "orbmi_matcher_destroy": (None, [_vp]),
    "orbmi_matcher_share_stream": (_i, [_vp, _vp]),
    "orbmi_matcher_get_stream": (_i, [_vp, C.POINTER(_vp)]),
    "orbmi_matcher_reserve_cus": (_i, [_vp, _i]),
    "orbmi_matcher_assign_features_to_grid": (_i, [_vp, _vp]),
    "orbmi_matcher_release_grid": (_i, [_vp]),
    "orbmi_matcher_build_grid_slot": (_i, [_vp, _vp, _i, _vp]),
    "orbmi_matcher_pin_grid_slot": (_i, [_vp, _vp, _i]),
    "orbmi_match_descriptors_segments": (_i, [_vp, _vp, _i, _vp, _vp, _i, _i, _vp, _i, _i, _f, _vp, _vp]),
    "orbmi_extractor_get_stream": (_i, [_vp, C.POINTER(_vp)]),
    "orbmi_is_in_frustum": (_i, [_vp, _vp, _vp, _i, _f, _vp]),
    "orbmi_search_by_projection_local": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _f, _f, _vp, C.POINTER(_i)]),
    "orbmi_search_local_points": (_i, [_vp, _vp, _vp, _vp, _i, _f, _vp, C.POINTER(_i), C.POINTER(_i)]),
    "orbmi_search_local_points_track": (_i, [_vp, _vp, _vp, _vp, _i, _f, _vp, C.POINTER(_i), C.POINTER(_i), _vp]),
    "orbmi_search_by_projection_last_frame": (_i, [_vp, _vp, _vp, _vp, _vp, _f, _i, _i, _vp, C.POINTER(_i)]),
    "orbmi_search_by_bow": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _f, _i, _vp, C.POINTER(_i)]),
    "orbmi_ba_create": (_i, [_i, C.POINTER(_vp)]),
    "orbmi_ba_destroy": (None, [_vp]),
    "orbmi_local_bundle_adjustment": (_i, [_vp, _vp, _vp, _vp]),
    "orbmi_pose_create": (_i, [_i, C.POINTER(_vp)]),
    "orbmi_pose_destroy": (None, [_vp]),
    "orbmi_pose_optimization": (_i, [_vp, _vp, _i, _vp, _i, _vp]),
    "orbmi_pose_synchronize": (_i, [_vp]),
    "orbmi_pose_share_stream": (_i, [_vp, _vp]),
    "orbmi_pose_share_matcher_stream": (_i, [_vp, _vp]),
    "orbmi_pose_set_profiling": (_i, [_vp, _i]),
    "orbmi_vocabulary_create": (_i, [_i, _vp, C.POINTER(_vp)]),
    "orbmi_vocabulary_destroy": (None, [_vp]),
    "orbmi_vocabulary_synchronize": (_i, [_vp]),
    "orbmi_vocabulary_share_stream": (_i, [_vp, _vp]),
    "orbmi_vocabulary_get_stream": (_i, [_vp, C.POINTER(_vp)]),
    "orbmi_transform": (_i, [_vp, _vp, _i, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp]),
    "orbmi_compute_distinctive_descriptors": (_i, [_vp, _vp, _vp, _i, _vp, _vp]),
    "orbmi_fuse_search": (_i, [_vp, _vp, _vp, _vp, _i, _f, _vp, _vp, C.POINTER(_i)]),
    "orbmi_search_for_triangulation": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp, C.POINTER(_i)]),
    "orbmi_search_for_triangulation_batch": (_i, [_vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _i, _i, _vp, _vp]),
    "orbmi_fuse_search_batch": (_i, [_vp, _i, _vp, _vp, _vp, _i, _f, _vp, _vp, _vp]),
    "orbmi_pose_read_profile": (_i, [_vp, _vp, _vp]),
    "orbmi_pose_optimization_frame": (_i, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "orbmi_pose_optimization_frame_track": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp]),
    "orbmi_search_by_projection_last_frame_if": (_i, [_vp, _vp, _vp, _vp, _vp, _f, _i, _i, _vp, _vp, _i]),
    "orbmi_track_update_matches": (_i, [_vp, _vp, _i, _vp, _vp, _vp, _vp]),
    "orbmi_set_profiling": (_i, [_vp, C.c_uint]),
    "orbmi_read_profile": (_i, [_vp, _vp, _vp]),
    "orbmi_debug_fast_candidates": (_i, [_vp, _i, _i, _vp, _i, C.POINTER(_i)]),
    "orbmi_debug_octree_level": (_i, [_vp, _i, _i, _vp, _i, C.POINTER(_i)]),
    "orbmi_debug_pose_trace": (_i, [_vp, _vp, _vp, _vp, _vp]),
    "orbmi_debug_greedy_stats": (_i, [_vp, _i]),
    "orbmi_debug_greedy_cycles": (_i, [_vp, _i]),
    "orbmi_compute_f12": (_i, [_vp, _vp, _vp]),
    "orbmi_triangulate_matches": (_i, [_vp, _vp, _vp, _vp, _i, _vp, _vp]),
    "orbmi_stereo_parallax_cos": (_i, [C.c_float, _vp, _i, _vp]),
    "orbmi_ba_set_stream": (_i, [_vp, _vp]),
    "orbmi_ba_set_stop_at_check": (_i, [_vp, _i]),
    "orbmi_ba_set_enqueued_hook": (_i, [_vp, _vp, _vp]),
    "orbmi_debug_ba_schur_blocks": (_i, [_i, _vp, _i, _vp]),
    "orbmi_vocabulary_set_stream": (_i, [_vp, _vp]),
    "orbmi_fuse_search_refresh": (_i, [_vp, _vp, _vp, _i, _vp, _vp, _i, _vp, _vp, _vp, _vp, _i, C.c_float, _vp, _vp]),
    "orbmi_create_new_map_points": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                         _vp]),
    "orbmi_slam_create": (_i, [_vp, _i, _vp, C.POINTER(_vp)]),
    "orbmi_slam_destroy": (None, [_vp]),
    "orbmi_slam_wait_local_mapping": (_i, [_vp]),
    "orbmi_slam_get_phase_ms": (_i, [_vp, _vp, _i, C.POINTER(C.c_long)]),
    "orbmi_slam_track_stereo": (_i, [_vp, _vp, _vp, _i, _i, _sz, C.c_double, _vp, C.POINTER(_i)]),
    "orbmi_slam_track_stereo_ahead": (_i, [_vp, _vp, _vp, _i, _i, _sz, C.c_double, _vp, _vp, _vp, C.POINTER(_i)]),
    "orbmi_slam_get_stats": (_i, [_vp, _i, _vp]),
    "orbmi_slam_get_schedule": (_i, [_vp, _vp, _i, C.POINTER(_i)]),
    "orbmi_slam_get_local_ba_log": (_i, [_vp, _vp, _i, C.POINTER(_i)]),
    "orbmi_slam_get_keyframe_state_log": (_i, [_vp, _vp, _i, C.POINTER(_i)]),
    "orbmi_slam_set_recording": (_i, [_vp, _i]),
    "orbmi_slam_get_local_mapping_counts": (_i, [_vp, _vp, _i]),
    "orbmi_slam_get_counts": (_i, [_vp, C.POINTER(_i), C.POINTER(_i), C.POINTER(_i), C.POINTER(_i)]),
    "orbmi_slam_get_trajectory": (_i, [_vp, _vp, _vp, _vp, _i, C.POINTER(_i)]),
    "orbmi_slam_save_trajectory_kitti": (_i, [_vp, C.c_char_p]),
    "orbmi_slam_save_trajectory_tum": (_i, [_vp, C.c_char_p]),
    "orbmi_slam_save_keyframe_trajectory_tum": (_i, [_vp, C.c_char_p]),
}

_lib = None


def lib() -> C.CDLL:
    """Load liborbmi.so (raises if it is absent: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        path = os.environ.get("ORBMI_LIB", LIB)  # an alternative build (A/B timing)
        if not os.path.exists(path):
            raise ImportError(f"{path} not built: run `python -m orb_slam2_with_comment_amd.build`")
        # torch bundles its own libamdhip64.so.7; loading it first lets liborbmi.so bind to that
        # same runtime (same SONAME) so torch tensors/streams/RCCL and our kernels share one HIP
        # runtime in the process.  Without torch, liborbmi.so uses /opt/rocm's runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(path)
        for name, (res, args) in _PROTOS.items():
            if os.environ.get("ORBMI_LIB") and not hasattr(L, name):  # an A/B build may predate an entry point
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(func: str, rc: int) -> None:
    if rc != ORBMI_OK:
        raise OrbmiError(func, rc)


def ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def declared_symbols(header: str | None = None):
    """Function names declared in include/orbmi*.h (used by the symbol-export test)."""
    import glob
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    names = []
    for h in ([header] if header else sorted(glob.glob(os.path.join(root, "include", "orbmi*.h")))):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names += re.findall(r"^\s*(?:int|void|float|double|const char\s*\*)\s+(orbmi_\w+)\s*\(", text, flags=re.M)
    return names
