"""numpy / ctypes mirrors of the C-ABI boundary structs (include/orbmi.h)."""
from __future__ import annotations

import ctypes as C

import numpy as np

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

# orbmi_mappoint
MAPPOINT_DTYPE = np.dtype([("pos", "<f4", 3), ("normal", "<f4", 3), ("max_distance", "<f4"),
                           ("min_distance", "<f4"), ("flags", "<u4"), ("desc", "u1", 32)])
# orbmi_mappoint_track
TRACK_DTYPE = np.dtype([("in_view", "<i4"), ("proj_x", "<f4"), ("proj_xr", "<f4"), ("proj_y", "<f4"),
                        ("level", "<i4"), ("view_cos", "<f4")])
# orbmi_lastframe_point
LFPOINT_DTYPE = np.dtype([("pos", "<f4", 3), ("flags", "<u4"), ("desc", "u1", 32)])

assert MAPPOINT_DTYPE.itemsize == 68 and TRACK_DTYPE.itemsize == 24 and LFPOINT_DTYPE.itemsize == 48

MP_BAD, MP_SEEN, MP_HAS_OBS = 1, 2, 4
LF_HAS_MP, LF_OUTLIER = 1, 2
FRAME_GRID_COLS, FRAME_GRID_ROWS = 64, 48


class FrameView(C.Structure):
    _fields_ = [("n", C.c_int), ("keys_un", C.c_void_p), ("u_right", C.c_void_p), ("desc", C.c_void_p),
                ("tcw", C.c_void_p), ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float),
                ("cy", C.c_float), ("bf", C.c_float), ("mb", C.c_float), ("min_x", C.c_float),
                ("max_x", C.c_float), ("min_y", C.c_float), ("max_y", C.c_float),
                ("grid_w_inv", C.c_float), ("grid_h_inv", C.c_float), ("nlevels", C.c_int),
                ("scale_factors", C.c_void_p), ("log_scale_factor", C.c_float), ("n_device", C.c_void_p)]


class VocabularyDesc(C.Structure):
    """orbmi_vocabulary_desc (include/orbmi.h): DBoW2::TemplatedVocabulary as flat arrays."""
    _fields_ = [("k", C.c_int), ("L", C.c_int), ("scoring", C.c_int), ("weighting", C.c_int), ("nnodes", C.c_int),
                ("desc", C.c_void_p), ("child_off", C.c_void_p), ("children", C.c_void_p), ("word_id", C.c_void_p),
                ("weight", C.c_void_p)]


class FeatureVectorView(C.Structure):
    _fields_ = [("nnodes", C.c_int), ("node_id", C.c_void_p), ("off", C.c_void_p), ("feat", C.c_void_p)]


class Frame:
    """Host-side Frame data the matchers read (include/Frame.h), kept alive for the views."""

    def __init__(self, keys, desc, u_right=None, tcw=None, cam=None, scale_factors=None, width=None,
                 height=None):
        self.keys = np.ascontiguousarray(keys, KP_DTYPE)
        self.desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        self.u_right = None if u_right is None else np.ascontiguousarray(u_right, np.float32)
        self.tcw = np.ascontiguousarray(np.eye(4) if tcw is None else tcw, np.float32)
        self.cam = cam
        sf = np.float32(1.2)
        if scale_factors is None:
            s, scale_factors = np.float32(1), []
            for _ in range(8):
                scale_factors.append(s)
                s = np.float32(np.float64(s) * np.float64(sf))
        self.scale_factors = np.ascontiguousarray(scale_factors, np.float32)
        self.width = width if width is not None else cam.width
        self.height = height if height is not None else cam.height

    def view(self) -> FrameView:
        v = FrameView()
        v.n = len(self.keys)
        v.keys_un = self.keys.ctypes.data
        v.u_right = self.u_right.ctypes.data if self.u_right is not None else None
        v.desc = self.desc.ctypes.data
        v.tcw = self.tcw.ctypes.data
        c = self.cam
        v.fx, v.fy, v.cx, v.cy, v.bf = c.fx, c.fy, c.cx, c.cy, c.bf
        v.mb = np.float32(np.float32(c.bf) / np.float32(c.fx))
        # ComputeImageBounds without distortion (src/Frame.cc:481-498)
        v.min_x, v.max_x, v.min_y, v.max_y = 0.0, float(self.width), 0.0, float(self.height)
        v.grid_w_inv = np.float32(np.float32(FRAME_GRID_COLS) / np.float32(self.width))
        v.grid_h_inv = np.float32(np.float32(FRAME_GRID_ROWS) / np.float32(self.height))
        v.nlevels = len(self.scale_factors)
        v.scale_factors = self.scale_factors.ctypes.data
        v.log_scale_factor = np.float32(np.log(np.float32(self.scale_factors[1]))) if len(self.scale_factors) > 1 else 0.0
        self._view = v
        return v


class FeatureVector:
    """DBoW2::FeatureVector as CSR (node ids ascending, features in insertion order)."""

    def __init__(self, node_of_feature: np.ndarray):
        node_of_feature = np.asarray(node_of_feature, np.int64)
        nodes = np.unique(node_of_feature)
        order = np.argsort(node_of_feature, kind="stable")
        counts = np.array([np.sum(node_of_feature == n) for n in nodes], np.int32)
        self.node_id = nodes.astype(np.uint32)
        self.off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
        self.feat = order.astype(np.int32)

    @classmethod
    def from_csr(cls, node_id, off, feat) -> "FeatureVector":
        """From CSR arrays (the output of ORBVocabulary.transform / orbmi_transform)."""
        fv = cls.__new__(cls)
        fv.node_id = np.ascontiguousarray(node_id, np.uint32)
        fv.off = np.ascontiguousarray(off, np.int32)
        fv.feat = np.ascontiguousarray(feat, np.int32)
        return fv

    def view(self) -> FeatureVectorView:
        v = FeatureVectorView()
        v.nnodes = len(self.node_id)
        v.node_id = self.node_id.ctypes.data
        v.off = self.off.ctypes.data
        v.feat = self.feat.ctypes.data
        self._view = v
        return v


# Optimizer::LocalBundleAdjustment boundary (orbmi_ba_* in include/orbmi.h)
BA_KF_DTYPE = np.dtype([("tcw", "<f4", 16), ("id", "<u4"), ("fixed", "<i4"), ("fx", "<f4"), ("fy", "<f4"),
                        ("cx", "<f4"), ("cy", "<f4"), ("bf", "<f4")])
BA_PT_DTYPE = np.dtype([("pos", "<f4", 3), ("id", "<u4"), ("bad", "<i4")])
BA_EDGE_DTYPE = np.dtype([("point", "<i4"), ("kf", "<i4"), ("u", "<f4"), ("v", "<f4"), ("ur", "<f4"),
                          ("inv_sigma2", "<f4")])
assert BA_KF_DTYPE.itemsize == 92 and BA_PT_DTYPE.itemsize == 20 and BA_EDGE_DTYPE.itemsize == 24


# orbmi_pose_obs / orbmi_pose_frame (Optimizer::PoseOptimization)
POSE_OBS_DTYPE = np.dtype([("Xw", "<f4", 3), ("u", "<f4"), ("v", "<f4"), ("ur", "<f4"), ("inv_sigma2", "<f4"),
                           ("index", "<i4")])
POSE_FRAME_DTYPE = np.dtype([("tcw", "<f4", 16), ("fx", "<f4"), ("fy", "<f4"), ("cx", "<f4"), ("cy", "<f4"),
                             ("bf", "<f4"), ("obs_begin", "<i4"), ("n_obs", "<i4"), ("inliers", "<i4"),
                             ("iterations", "<i4")])
assert POSE_OBS_DTYPE.itemsize == 32 and POSE_FRAME_DTYPE.itemsize == 100


class TriKeyFrame(C.Structure):
    """orbmi_tri_keyframe: the KeyFrame members CreateNewMapPoints reads (include/orbmi.h)."""
    _fields_ = [("tcw", C.c_void_p), ("keys_un", C.c_void_p), ("u_right", C.c_void_p), ("depth", C.c_void_p),
                ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float),
                ("mb", C.c_float), ("level_sigma2", C.c_void_p), ("scale_factors", C.c_void_p)]


class FrameMapPoints(C.Structure):
    """orbmi_frame_mappoints: Frame::mvpMapPoints as match arrays (include/orbmi.h)."""
    _fields_ = [("match_lf", C.c_void_p), ("lf_points", C.c_void_p), ("n_lf_points", C.c_int),
                ("match_mp", C.c_void_p), ("mps", C.c_void_p), ("n_mps", C.c_int)]


class BAProblemView(C.Structure):
    _fields_ = [("nkf", C.c_int), ("npt", C.c_int), ("nedge", C.c_int), ("kfs", C.c_void_p), ("pts", C.c_void_p),
                ("edges", C.c_void_p)]


class BAResultView(C.Structure):
    _fields_ = [("tcw", C.c_void_p), ("pos", C.c_void_p), ("erase", C.c_void_p), ("iterations", C.c_int * 2),
                ("chi2", C.c_double * 2), ("aborted", C.c_int), ("stop_check", C.c_int), ("checks", C.c_int)]


class BAProblem:
    """Local-BA graph as the C ABI takes it; keeps arrays alive for the views."""

    def __init__(self, kfs, pts, edges):
        self.kfs = np.ascontiguousarray(kfs, BA_KF_DTYPE)
        self.pts = np.ascontiguousarray(pts, BA_PT_DTYPE)
        self.edges = np.ascontiguousarray(edges, BA_EDGE_DTYPE)

    def view(self):
        v = BAProblemView(len(self.kfs), len(self.pts), len(self.edges), self.kfs.ctypes.data, self.pts.ctypes.data,
                          self.edges.ctypes.data)
        self._v = v
        return v

    def result_buffers(self):
        tcw = np.zeros((max(len(self.kfs), 1), 16), np.float32)
        pos = np.zeros((max(len(self.pts), 1), 3), np.float32)
        erase = np.zeros(max(len(self.edges), 1), np.uint8)
        r = BAResultView(tcw.ctypes.data, pos.ctypes.data, erase.ctypes.data)
        return r, tcw, pos, erase
