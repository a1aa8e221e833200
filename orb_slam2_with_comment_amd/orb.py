"""Python mirror of the reference's ORB front-end interface, over the C ABI (liborbmi.so).

`ORBextractor` mirrors include/ORBextractor.h:45-111 (constructor arguments, operator(),
getters, mvImagePyramid); `compute_stereo_matches` mirrors Frame::ComputeStereoMatches
(src/Frame.cc:501-675).  Every call runs the hand-written HIP kernels; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _capi
from ._capi import KP_DTYPE, check, lib, ptr


class ORBextractor:
    """ORB_SLAM2::ORBextractor on one MI355X (include/ORBextractor.h:58-59)."""

    def __init__(self, nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int,
                 minThFAST: int, device: int = 0):
        h = C.c_void_p()
        check("orbmi_extractor_create",
              lib().orbmi_extractor_create(device, nfeatures, scaleFactor, nlevels, iniThFAST,
                                           minThFAST, C.byref(h)))
        self._h = h
        self.nfeatures = nfeatures
        self.nlevels = nlevels
        self.device = device
        self._shape = None

    def close(self):
        if getattr(self, "_h", None):
            lib().orbmi_extractor_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # ORBextractor::operator()(image, mask, keypoints, descriptors)  src/ORBextractor.cc:1043
    def __call__(self, image: np.ndarray, mask=None):
        """Returns (keypoints [structured KP_DTYPE], descriptors [n x 32 u8] or None).

        The mask is ignored, as in the reference (include/ORBextractor.h:62-63)."""
        image = np.asarray(image)
        if image.size == 0:
            return np.zeros(0, KP_DTYPE), None
        if image.dtype != np.uint8 or image.ndim != 2:
            raise TypeError("ORBextractor expects a CV_8UC1 image (src/ORBextractor.cc:1050)")
        image = np.ascontiguousarray(image)
        cap = self.nfeatures + 16 * self.nlevels + 64
        while True:
            kps = np.zeros(cap, KP_DTYPE)
            desc = np.zeros((cap, 32), np.uint8)
            n = C.c_int()
            rc = lib().orbmi_extract(self._h, ptr(image), image.shape[0], image.shape[1],
                                     image.strides[0], ptr(kps), ptr(desc), cap, C.byref(n))
            if rc == _capi.ORBMI_E_CAP:
                cap = n.value
                continue
            check("orbmi_extract", rc)
            break
        self._shape = image.shape
        n = n.value
        if n == 0:
            return kps[:0].copy(), None  # descriptors.release() (src/ORBextractor.cc:1063-1064)
        return kps[:n].copy(), desc[:n].copy()

    def _levels_f(self, fn):
        out = np.zeros(self.nlevels, np.float32)
        check(fn, getattr(lib(), fn)(self._h, ptr(out)))
        return out

    def GetLevels(self) -> int:
        return lib().orbmi_extractor_get_levels(self._h)

    def GetScaleFactor(self) -> float:
        return lib().orbmi_extractor_get_scale_factor(self._h)

    def GetScaleFactors(self):
        return self._levels_f("orbmi_extractor_get_scale_factors")

    def GetInverseScaleFactors(self):
        return self._levels_f("orbmi_extractor_get_inverse_scale_factors")

    def GetScaleSigmaSquares(self):
        return self._levels_f("orbmi_extractor_get_scale_sigma_squares")

    def GetInverseScaleSigmaSquares(self):
        return self._levels_f("orbmi_extractor_get_inverse_scale_sigma_squares")

    def features_per_level(self):
        out = np.zeros(self.nlevels, np.int32)
        check("orbmi_extractor_get_features_per_level",
              lib().orbmi_extractor_get_features_per_level(self._h, ptr(out)))
        return out

    def pyramid_level(self, level: int, padded: bool = False, item: int = 0) -> np.ndarray:
        """mvImagePyramid[level] of the last extraction (padded: with the 19-px border)."""
        rows, cols = self._shape if self._shape else (4096, 4096)
        cap_w, cap_h = cols + 64, rows + 64
        out = np.zeros((cap_h, cap_w), np.uint8)
        w, h = C.c_int(), C.c_int()
        check("orbmi_extractor_get_pyramid_level",
              lib().orbmi_extractor_get_pyramid_level(self._h, item, level, int(padded), ptr(out),
                                                      cap_w, C.byref(w), C.byref(h)))
        return out[:h.value, :w.value].copy()

    @property
    def mvImagePyramid(self):
        return [self.pyramid_level(l) for l in range(self.nlevels)]


def compute_stereo_matches(left: ORBextractor, right: ORBextractor, bf: float, fx: float,
                           n_left: int, item_left: int = 0, item_right: int = 0):
    """Frame::ComputeStereoMatches (src/Frame.cc:501-675) on the last extractions of
    `left` and `right`; returns (mvuRight, mvDepth) float32 arrays of n_left entries."""
    u = np.full(max(n_left, 1), -1, np.float32)
    d = np.full(max(n_left, 1), -1, np.float32)
    check("orbmi_compute_stereo_matches",
          lib().orbmi_compute_stereo_matches(left.handle, item_left, right.handle, item_right, bf, fx,
                                             ptr(u), ptr(d), n_left))
    return u[:n_left], d[:n_left]
