"""Python mirror of ORB_SLAM2::ORBmatcher (include/ORBmatcher.h:37-102) over the C ABI.

The map/frame state crosses the boundary as flat arrays (types.py): keypoints, descriptors,
mvuRight and the pose of a Frame; MapPoint state as orbmi_mappoint records.  Results are the
reference's side effects as index arrays (see include/orbmi.h for the codes)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._capi import check, lib
from .types import TRACK_DTYPE


class ORBmatcher:
    TH_HIGH, TH_LOW, HISTO_LENGTH = 100, 50, 30  # src/ORBmatcher.cc:37-39

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, device: int = 0):
        h = C.c_void_p()
        check("orbmi_matcher_create", lib().orbmi_matcher_create(device, C.byref(h)))
        self._h = h
        self.mfNNratio = nnratio
        self.mbCheckOrientation = checkOri

    def close(self):
        if getattr(self, "_h", None):
            lib().orbmi_matcher_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def IsInFrustum(self, frame, mps, viewing_cos_limit=0.5):
        """Frame::isInFrustum over all points (src/Frame.cc:274-342)."""
        mps = np.ascontiguousarray(mps)
        tr = np.zeros(max(len(mps), 1), TRACK_DTYPE)
        v = frame.view()
        check("orbmi_is_in_frustum", lib().orbmi_is_in_frustum(self._h, C.addressof(v), mps.ctypes.data, len(mps),
                                                               viewing_cos_limit, tr.ctypes.data))
        return tr[:len(mps)]

    def SearchByProjection(self, frame, occupied, mps, track, th=3.0):
        """SearchByProjection(Frame&, vector<MapPoint*>, th) (src/ORBmatcher.cc:59-155)."""
        occ = np.ascontiguousarray(occupied, np.uint8)
        mps = np.ascontiguousarray(mps)
        track = np.ascontiguousarray(track)
        out = np.zeros(max(len(frame.keys), 1), np.int32)
        n = C.c_int()
        v = frame.view()
        check("orbmi_search_by_projection_local",
              lib().orbmi_search_by_projection_local(self._h, C.addressof(v), occ.ctypes.data, mps.ctypes.data,
                                                     track.ctypes.data, len(mps), th, self.mfNNratio,
                                                     out.ctypes.data, C.byref(n)))
        return out[:len(frame.keys)], n.value

    def SearchLocalPoints(self, frame, occupied, mps, th=1.0):
        """Tracking::SearchLocalPoints (src/Tracking.cc:1345-1403) fused on the GPU."""
        occ = np.ascontiguousarray(occupied, np.uint8)
        mps = np.ascontiguousarray(mps)
        out = np.zeros(max(len(frame.keys), 1), np.int32)
        n, ntm = C.c_int(), C.c_int()
        v = frame.view()
        check("orbmi_search_local_points",
              lib().orbmi_search_local_points(self._h, C.addressof(v), occ.ctypes.data, mps.ctypes.data, len(mps), th,
                                              out.ctypes.data, C.byref(n), C.byref(ntm)))
        return out[:len(frame.keys)], n.value, ntm.value

    def SearchByProjectionLastFrame(self, cf, occupied, lf, lf_points, th, bMono=False):
        """SearchByProjection(Frame& CF, const Frame& LF, th, bMono) (src/ORBmatcher.cc:1540-1695)."""
        occ = np.ascontiguousarray(occupied, np.uint8)
        lfp = np.ascontiguousarray(lf_points)
        out = np.zeros(max(len(cf.keys), 1), np.int32)
        n = C.c_int()
        vc, vl = cf.view(), lf.view()
        check("orbmi_search_by_projection_last_frame",
              lib().orbmi_search_by_projection_last_frame(self._h, C.addressof(vc), occ.ctypes.data, C.addressof(vl),
                                                          lfp.ctypes.data, th, int(bMono),
                                                          int(self.mbCheckOrientation), out.ctypes.data, C.byref(n)))
        return out[:len(cf.keys)], n.value

    def SearchForTriangulation(self, kf1, has_mp1, fv1, kf2, has_mp2, fv2, F12, bOnlyStereo=False):
        """SearchForTriangulation(KeyFrame*, KeyFrame*, cv::Mat F12, vector<pair<size_t,size_t>>&,
        bool) (src/ORBmatcher.cc:783-975): kf1 / kf2 are types.Frame (keys_un, u_right, desc, tcw),
        has_mp = GetMapPoint(i) != NULL, fv = mFeatVec.  Returns (match12, nmatches); the matched
        pairs are (i, match12[i]) for match12[i] >= 0."""
        m1 = np.ascontiguousarray(has_mp1, np.uint8)
        m2 = np.ascontiguousarray(has_mp2, np.uint8)
        F = np.ascontiguousarray(F12, np.float32).reshape(3, 3)
        out = np.zeros(max(len(kf1.keys), 1), np.int32)
        n = C.c_int()
        v1, v2, f1, f2 = kf1.view(), kf2.view(), fv1.view(), fv2.view()
        check("orbmi_search_for_triangulation", lib().orbmi_search_for_triangulation(
            self._h, C.addressof(v1), m1.ctypes.data, C.addressof(f1), C.addressof(v2), m2.ctypes.data,
            C.addressof(f2), F.ctypes.data, int(bOnlyStereo), int(self.mbCheckOrientation), out.ctypes.data,
            C.byref(n)))
        return out[:len(kf1.keys)], n.value

    def FuseSearch(self, kf, mps, in_kf=None, th=3.0):
        """The search of Fuse(KeyFrame*, const vector<MapPoint*>&, th) (src/ORBmatcher.cc:977-1127):
        -> (best_idx, best_dist, ncandidates); the Replace / AddObservation replay in list order
        is the caller's (include/orbmi.h)."""
        mps = np.ascontiguousarray(mps)
        n = len(mps)
        ink = None if in_kf is None else np.ascontiguousarray(in_kf, np.uint8)
        bi, bd = np.zeros(max(n, 1), np.int32), np.zeros(max(n, 1), np.int32)
        c = C.c_int()
        v = kf.view()
        check("orbmi_fuse_search", lib().orbmi_fuse_search(
            self._h, C.addressof(v), mps.ctypes.data if n else None, None if ink is None else ink.ctypes.data, n,
            th, bi.ctypes.data, bd.ctypes.data, C.byref(c)))
        return bi[:n], bd[:n], c.value

    def ComputeDistinctiveDescriptors(self, obs_desc: np.ndarray, obs_off: np.ndarray, desc_out=None):
        """MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:247-316) for a batch of map
        points: rows obs_off[p]..obs_off[p+1] of obs_desc are point p's observation descriptors.
        Returns (best row per point, -1 without observations; np x 32 mDescriptor)."""
        d = np.ascontiguousarray(obs_desc, np.uint8).reshape(-1, 32)
        off = np.ascontiguousarray(obs_off, np.int32)
        n = len(off) - 1
        best = np.zeros(max(n, 1), np.int32)
        out = np.zeros((max(n, 1), 32), np.uint8) if desc_out is None else np.ascontiguousarray(desc_out, np.uint8)
        check("orbmi_compute_distinctive_descriptors", lib().orbmi_compute_distinctive_descriptors(
            self._h, d.ctypes.data if len(d) else None, off.ctypes.data, n, best.ctypes.data, out.ctypes.data))
        return best[:n], out[:n]

    def SearchByBoW(self, kf, kf_mp_ok, kf_fv, f, f_fv):
        """SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) (src/ORBmatcher.cc:211-344)."""
        ok = np.ascontiguousarray(kf_mp_ok, np.uint8)
        out = np.zeros(max(len(f.keys), 1), np.int32)
        n = C.c_int()
        vk, vf, fk, ff = kf.view(), f.view(), kf_fv.view(), f_fv.view()
        check("orbmi_search_by_bow",
              lib().orbmi_search_by_bow(self._h, C.addressof(vk), ok.ctypes.data, C.addressof(fk), C.addressof(vf),
                                        C.addressof(ff), self.mfNNratio, int(self.mbCheckOrientation),
                                        out.ctypes.data, C.byref(n)))
        return out[:len(f.keys)], n.value
