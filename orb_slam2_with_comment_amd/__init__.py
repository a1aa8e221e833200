"""orb_slam2_with_comment_amd — MI355X-native ORB front-end and local BA for ORB-SLAM2.

The hot path of AHzZ123/orb_slam2_with_comment as hand-written HIP kernels
for gfx950 behind a C ABI (include/orbmi.h, liborbmi.so).  This package holds the kernels
(csrc/), their build (build.py), the ctypes binding (_capi.py) and a Python mirror of the
reference interface (orb.py) used by tests and bench.py.
"""
from .matcher import ORBmatcher  # noqa: F401
from .orb import ORBextractor, compute_stereo_matches  # noqa: F401

__all__ = ["ORBextractor", "ORBmatcher", "compute_stereo_matches"]
