"""Device-resident Track + LocalMap pipeline over the C ABI.

One tracked stereo frame, in the order Tracking runs it (src/Tracking.cc:287-581):

  Frame ctor          ORBextractor(left) || ORBextractor(right)   src/Frame.cc:78-81
                      Frame::ComputeStereoMatches                 src/Frame.cc:92
  TrackWithMotionModel ORBmatcher(0.9).SearchByProjection(CF, LF, th=7) [+ retry at 14 when
                      < 20 matches], Optimizer::PoseOptimization, discard outliers
                                                                  src/Tracking.cc:997-1063
  TrackLocalMap       Tracking::SearchLocalPoints -> isInFrustum(0.5) +
                      ORBmatcher(0.8).SearchByProjection(F, localMPs, th=1) at the optimised
                      pose, Optimizer::PoseOptimization, mnMatchesInliers
                                                                  src/Tracking.cc:1065-1104
  LocalMapping thread KeyFrame::ComputeBoW + Optimizer::LocalBundleAdjustment on every new
                      keyframe (src/LocalMapping.cc:89-90, :152-160), concurrently with tracking

The tracking stages run on one HIP stream (the matcher's; the pose optimiser shares it) and the
Frame constructor's extraction on the extractor's stream, double-buffered, so that the next
frame's extraction overlaps this frame's tracking (StereoTracker(pipelined=True); with
pipelined=False everything shares the extractor's stream).  Inputs and outputs stay in HBM,
keypoint counts are read on the device (orbmi_frame_view.n_device) and the optimised pose is
read by the next search from its device record (orbmi_frame_view.tcw in device memory), so a
frame is enqueued without a host round trip.  Local BA runs on its own stream from a worker thread (the LocalMapping thread),
overlapping tracking as in the reference.
"""
from __future__ import annotations

import ctypes as C
import os
import queue
import threading
import time

import numpy as np

from . import _capi
from ._capi import check, lib
from ._hip import PinnedWords
from .types import FRAME_GRID_COLS, FRAME_GRID_ROWS, FrameView

_vp = C.c_void_p


def frame_view(n, keys, u_right, desc, tcw, cam, scale_factors, width, height, n_device=None):
    """orbmi_frame_view over (device or host) addresses; tcw / scale_factors are numpy arrays
    that must outlive the view."""
    v = FrameView()
    v.n = int(n)
    v.keys_un, v.u_right, v.desc = keys, u_right, desc
    v.tcw = tcw.ctypes.data if isinstance(tcw, np.ndarray) else None
    v.fx, v.fy, v.cx, v.cy, v.bf = cam.fx, cam.fy, cam.cx, cam.cy, cam.bf
    v.mb = np.float32(np.float32(cam.bf) / np.float32(cam.fx))
    v.min_x, v.max_x, v.min_y, v.max_y = 0.0, float(width), 0.0, float(height)
    v.grid_w_inv = np.float32(np.float32(FRAME_GRID_COLS) / np.float32(width))
    v.grid_h_inv = np.float32(np.float32(FRAME_GRID_ROWS) / np.float32(height))
    v.nlevels = len(scale_factors)
    v.scale_factors = scale_factors.ctypes.data
    v.log_scale_factor = np.float32(np.log(np.float32(scale_factors[1]))) if len(scale_factors) > 1 else 0.0
    v.n_device = n_device
    if isinstance(tcw, int):  # device address (an orbmi_pose_frame record's tcw)
        v.tcw = tcw
    return v


class StereoTracker:
    """Tracking-thread GPU work for one stereo stream (one GPU).

    pipelined=False: extraction, searches and pose optimisations run on ONE stream (the
    extractor's).  pipelined=True: the Frame constructor's work (extraction + stereo) runs on the
    extractor's stream E and the tracking stages on the matcher's stream T, with the frame
    buffers double-buffered in two slots, so frame k+1's extraction overlaps frame k's tracking
    (it depends only on the image; the reference builds the Frame before Track() too,
    src/Tracking.cc:168-205).  Frame k's tracking waits for its own extraction (event), and
    frame k+2's extraction for frame k's tracking to release the slot."""

    def __init__(self, cam, nfeatures=2000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7, device=0,
                 pipelined=False):
        import torch
        from .matcher import ORBmatcher
        from .optimizer import PoseOptimizer
        from .orb import ORBextractor
        from .types import POSE_FRAME_DTYPE
        self.cam, self.device, self.pipelined = cam, device, pipelined
        self.unfused = os.environ.get("ORBMI_TRACK_UNFUSED") == "1"  # A/B: pose and update as two launches
        # ORBMI_GRID_AHEAD=1 (pipelined): Frame::AssignFeaturesToGrid on the extraction stream
        # right after the frame's keypoints (a slot grid per frame slot), off the tracking chain.
        # Tracking alone gains 3.5 % (0.319 -> 0.308 ms per frame back to back), but the headline
        # with the concurrent LocalMapping chain loses 2.7 % (profiles/r06/grid_ahead_ab.txt), so
        # the default builds the grid on the tracking stream at the first search
        self.grid_ahead = pipelined and os.environ.get("ORBMI_GRID_AHEAD", "0") == "1"
        self._tcw0 = np.eye(4, dtype=np.float32)  # (the grid reads no pose)
        self.frame_events = None  # a list: per-frame [extract start, end, track start, end] events (pipelined)
        self.extractor = ORBextractor(nfeatures, scale_factor, nlevels, ini_th, min_th, device=device)
        self.matcher = ORBmatcher(device=device)
        self.pose = PoseOptimizer(device)
        L = lib()
        if pipelined:
            check("orbmi_pose_share_matcher_stream", L.orbmi_pose_share_matcher_stream(self.pose._h, self.matcher._h))
        else:
            check("orbmi_matcher_share_stream", L.orbmi_matcher_share_stream(self.matcher._h, self.extractor.handle))
            self.pose.share_stream(self.extractor.handle)
        self.inv_sigma2 = np.ascontiguousarray(self.extractor.GetInverseScaleSigmaSquares(), np.float32)
        s = _vp()
        check("orbmi_extractor_get_stream", L.orbmi_extractor_get_stream(self.extractor.handle, C.byref(s)))
        self.stream_handle = s.value  # extraction stream E
        t = _vp()
        check("orbmi_matcher_get_stream", L.orbmi_matcher_get_stream(self.matcher._h, C.byref(t)))
        self.track_stream_handle = t.value  # tracking stream T (== E unless pipelined)
        self.scale_factors = self.extractor.GetScaleFactors()
        self.cap = cap = nfeatures + 64
        dev = torch.device("cuda", device)
        nslots = 2 if pipelined else 1
        # per slot: outputs of a frame's extraction (item 0 = left, 1 = right)
        self.slots = [dict(kps=torch.zeros((2, cap, 7), dtype=torch.int32, device=dev),
                           desc=torch.zeros((2, cap, 32), dtype=torch.uint8, device=dev),
                           counts=torch.zeros(2, dtype=torch.int32, device=dev),
                           u_right=torch.zeros((2, cap), dtype=torch.float32, device=dev),
                           depth=torch.zeros((2, cap), dtype=torch.float32, device=dev)) for _ in range(nslots)]
        self.slot = 0        # slot of the frame tracked last (the kps/desc/... properties)
        self._next = 0       # slot of the next frame
        if pipelined:
            self._E = torch.cuda.ExternalStream(self.stream_handle, device=dev)
            self._T = torch.cuda.ExternalStream(self.track_stream_handle, device=dev)
            self._ev_extracted = [torch.cuda.Event() for _ in range(nslots)]
            self._ev_tracked = [torch.cuda.Event() for _ in range(nslots)]
            self._pending = [False] * nslots
            self._holds = [[] for _ in range(nslots)]  # other consumers' events per slot (hold_slot)
        self.occupied = torch.zeros(cap, dtype=torch.uint8, device=dev)   # after the motion-model stage
        self.no_points = torch.zeros(cap, dtype=torch.uint8, device=dev)  # fill(mvpMapPoints, NULL)
        self.match_lf = torch.full((cap,), -1, dtype=torch.int32, device=dev)
        self.match_mp = torch.full((cap,), -1, dtype=torch.int32, device=dev)
        self.outlier = torch.zeros(cap, dtype=torch.uint8, device=dev)    # mvbOutlier
        # pose records: [0] after TrackWithMotionModel, [1] after TrackLocalMap (POSE_FRAME_DTYPE)
        self.rec_bytes = POSE_FRAME_DTYPE.itemsize
        self.recs = torch.zeros((2, self.rec_bytes), dtype=torch.uint8, device=dev)
        # [0] SearchByProjection(CF, LF) matches, [1:3] stage-0 counts, [3:5] stage-1 counts
        self.tcounts = torch.zeros(8, dtype=torch.int32, device=dev)
        self._views = {}

    # the frame tracked last (its slot's buffers)
    kps = property(lambda self: self.slots[self.slot]["kps"])
    desc = property(lambda self: self.slots[self.slot]["desc"])
    counts = property(lambda self: self.slots[self.slot]["counts"])
    u_right = property(lambda self: self.slots[self.slot]["u_right"])
    depth = property(lambda self: self.slots[self.slot]["depth"])

    def rec_tcw(self, k):
        """Device address of pose record k's tcw (its first field)."""
        return self.recs.data_ptr() + k * self.rec_bytes

    def current_view(self, tcw):
        """Frame view of the frame being tracked (its slot's device arrays, device count); tcw =
        host numpy pose or the device address of a pose record."""
        key = (self.slot, tcw if isinstance(tcw, int) else tcw.ctypes.data)
        v = self._views.get(key)
        if v is None:
            sl = self.slots[self.slot]
            v = frame_view(self.cap, sl["kps"].data_ptr(), sl["u_right"].data_ptr(), sl["desc"].data_ptr(), tcw,
                           self.cam, self.scale_factors, self.cam.width, self.cam.height,
                           n_device=sl["counts"].data_ptr())
            self._views[key] = v
        return v

    def extract_stereo(self, d_left_right: int, rows: int, cols: int, slot=None, host=False):
        """ORBextractor(left) + ORBextractor(right) as one batch + ComputeStereoMatches into
        `slot` (default: the current one) on the extraction stream; d_left_right = device address
        of the 2 x rows x cols u8 image pair (host=True: host address, copied to HBM by the
        extraction stream itself, orbmi_extract_batch_host)."""
        L = lib()
        sl = self.slots[self.slot if slot is None else slot]
        if host:
            check("orbmi_extract_batch_host", L.orbmi_extract_batch_host(
                self.extractor.handle, _vp(d_left_right), 2, rows, cols, rows * cols, _vp(sl["kps"].data_ptr()),
                _vp(sl["desc"].data_ptr()), _vp(sl["counts"].data_ptr()), self.cap))
        else:
            check("orbmi_extract_batch_device", L.orbmi_extract_batch_device(
                self.extractor.handle, _vp(d_left_right), 2, rows, cols, cols, rows * cols, _vp(sl["kps"].data_ptr()),
                _vp(sl["desc"].data_ptr()), _vp(sl["counts"].data_ptr()), self.cap))
        check("orbmi_compute_stereo_matches_batch_device", L.orbmi_compute_stereo_matches_batch_device(
            self.extractor.handle, self.cam.bf, self.cam.fx, _vp(sl["u_right"].data_ptr()), _vp(sl["depth"].data_ptr())))
        # new keypoints behind the slot's pointers: a grid pinned on an earlier frame is stale
        check("orbmi_matcher_release_grid", L.orbmi_matcher_release_grid(self.matcher._h))
        if self.grid_ahead and slot is not None:
            # the slot's grid, in stream order behind its keypoints; the searches read it behind the
            # extraction event, and the slot's next extraction waits for them (_ev_tracked)
            v = frame_view(self.cap, sl["kps"].data_ptr(), sl["u_right"].data_ptr(), sl["desc"].data_ptr(), self._tcw0,
                           self.cam, self.scale_factors, self.cam.width, self.cam.height,
                           n_device=sl["counts"].data_ptr())
            check("orbmi_matcher_build_grid_slot", L.orbmi_matcher_build_grid_slot(
                self.matcher._h, C.addressof(v), int(slot), _vp(self.stream_handle)))

    def search_last_frame(self, tcw, last_view, last_points, th=7.0):
        """ORBmatcher(0.9, true).SearchByProjection(mCurrentFrame, mLastFrame, th, !stereo)
        (src/Tracking.cc:1016) -> self.match_lf (device)."""
        cv = self.current_view(tcw)
        check("orbmi_search_by_projection_last_frame", lib().orbmi_search_by_projection_last_frame(
            self.matcher._h, C.addressof(cv), _vp(self.no_points.data_ptr()), C.addressof(last_view),
            _vp(last_points), th, 0, 1, _vp(self.match_lf.data_ptr()), None))

    def search_local_points(self, tcw, local_mps, n_mp, th=1.0):
        """Tracking::SearchLocalPoints (src/Tracking.cc:1362-1402) -> self.match_mp (device)."""
        cv = self.current_view(tcw)
        check("orbmi_search_local_points", lib().orbmi_search_local_points(
            self.matcher._h, C.addressof(cv), _vp(self.occupied.data_ptr()), _vp(local_mps), int(n_mp), th,
            _vp(self.match_mp.data_ptr()), None, None))

    def track_with_motion_model(self, tcw, last_view, last_points, th=7.0):
        """Tracking::TrackWithMotionModel (src/Tracking.cc:997-1063) after the frame's
        extraction: SearchByProjection(CF, LF, th) from the motion-model pose `tcw` (host), the
        retry at 2*th when fewer than 20 matches (device-side test), PoseOptimization -> pose
        record 0, outliers discarded -> self.occupied for the local-map search."""
        L = lib()
        cv = self.current_view(tcw)
        # Frame::AssignFeaturesToGrid once per frame: both last-frame searches and the
        # local-map search reuse this grid (built ahead on the extraction stream when grid_ahead)
        if self.grid_ahead:
            check("orbmi_matcher_pin_grid_slot",
                  L.orbmi_matcher_pin_grid_slot(self.matcher._h, C.addressof(cv), int(self.slot)))
        else:
            check("orbmi_matcher_assign_features_to_grid",
                  L.orbmi_matcher_assign_features_to_grid(self.matcher._h, C.addressof(cv)))
        mp = self.frame_mappoints(last_view, last_points, None, 0)
        for t, gate in ((th, 0x7FFFFFFF), (2 * th, 20)):  # the first search always runs
            check("orbmi_search_by_projection_last_frame_if", L.orbmi_search_by_projection_last_frame_if(
                self.matcher._h, C.addressof(cv), _vp(self.no_points.data_ptr()), C.addressof(last_view),
                _vp(last_points), t, 0, 1, _vp(self.match_lf.data_ptr()), _vp(self.tcounts.data_ptr()), gate))
        self._pose_and_update(cv, mp, 0, 0, self.occupied.data_ptr(), self.tcounts.data_ptr() + 4)

    def track_local_map(self, last_view, last_points, local_mps, n_mp, th=1.0):
        """Tracking::TrackLocalMap (src/Tracking.cc:1065-1104) at pose record 0: SearchLocalPoints,
        PoseOptimization -> pose record 1, mnMatchesInliers (stereo outliers -> NULL)."""
        L = lib()
        cv = self.current_view(self.rec_tcw(0))
        check("orbmi_search_local_points", L.orbmi_search_local_points(
            self.matcher._h, C.addressof(cv), _vp(self.occupied.data_ptr()), _vp(local_mps), int(n_mp), th,
            _vp(self.match_mp.data_ptr()), None, None))
        mp = self.frame_mappoints(last_view, last_points, local_mps, n_mp)
        self._pose_and_update(cv, mp, 1, 1, None, self.tcounts.data_ptr() + 12)

    def _pose_and_update(self, cv, mp, rec, stage, occupied, counts):
        """PoseOptimization -> pose record `rec`, then Tracking's pass over mvpMapPoints (stage 0:
        TrackWithMotionModel's outlier discard, 1: TrackLocalMap's statistics), as one launch
        (orbmi_pose_optimization_frame_track); ORBMI_TRACK_UNFUSED=1 issues the two calls."""
        if not self.unfused:
            self.pose.PoseOptimizationTrack(cv, self.inv_sigma2, mp, self.rec_tcw(rec), self.outlier.data_ptr(), stage,
                                            occupied, counts)
            return
        self.pose.PoseOptimization(cv, self.inv_sigma2, mp, self.rec_tcw(rec), self.outlier.data_ptr())
        check("orbmi_track_update_matches", lib().orbmi_track_update_matches(
            self.matcher._h, C.addressof(cv), stage, _vp(self.outlier.data_ptr()), C.addressof(mp), _vp(occupied),
            _vp(counts)))

    def frame_mappoints(self, last_view, last_points, local_mps, n_mp):
        from .types import FrameMapPoints
        mp = FrameMapPoints()
        mp.match_lf, mp.lf_points, mp.n_lf_points = self.match_lf.data_ptr(), last_points, last_view.n
        if local_mps is not None:
            mp.match_mp, mp.mps, mp.n_mps = self.match_mp.data_ptr(), local_mps, int(n_mp)
        return mp

    def track(self, d_left_right, rows, cols, tcw, last_view, last_points, local_mps, n_mp, th_lf=7.0, th_local=1.0,
              host=False):
        """Enqueue one tracked stereo frame (Frame ctor + TrackWithMotionModel + TrackLocalMap);
        results stay on the device: self.match_lf / match_mp (final mvpMapPoints), self.outlier,
        pose records self.recs, counts self.tcounts (see results()).  host=True: d_left_right is
        a host pair (pinned: read in place), copied to HBM by the extraction stream ahead of its
        extraction (orbmi_extract_batch_host), so the copy of frame k+1 overlaps frame k's
        tracking as its extraction does."""
        if not self.pipelined:
            self.extract_stereo(d_left_right, rows, cols, host=host)
            self.track_with_motion_model(tcw, last_view, last_points, th_lf)
            self.track_local_map(last_view, last_points, local_mps, n_mp, th_local)
            return
        s = self._next
        self._next ^= 1
        if self._pending[s]:  # the slot's previous frame must be tracked before it is overwritten
            self._E.wait_event(self._ev_tracked[s])
        for ev in self._holds[s]:  # ... and read by every other consumer (hold_slot)
            self._E.wait_event(ev)
        self._holds[s].clear()
        fe = self.frame_events
        if fe is not None:  # diagnostics: extraction / tracking start and end on their streams
            import torch
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            ev[0].record(self._E)
        self.extract_stereo(d_left_right, rows, cols, slot=s, host=host)
        self._ev_extracted[s].record(self._E)
        if fe is not None:
            ev[1].record(self._E)
        self._T.wait_event(self._ev_extracted[s])
        if fe is not None:
            ev[2].record(self._T)
        self.slot = s
        self.track_with_motion_model(tcw, last_view, last_points, th_lf)
        self.track_local_map(last_view, last_points, local_mps, n_mp, th_local)
        self._ev_tracked[s].record(self._T)
        if fe is not None:
            ev[3].record(self._T)
            fe.append(ev)
        self._pending[s] = True

    def hold_slot(self, stream):
        """Register another reader of the last tracked frame's slot (e.g. the config-4 exchange
        on its own stream): the extraction that next overwrites the slot waits for the work
        enqueued on `stream` so far."""
        import torch
        ev = torch.cuda.Event()
        ev.record(stream)
        if self.pipelined:
            self._holds[self.slot].append(ev)
        else:  # one stream: the next extraction is on E
            torch.cuda.ExternalStream(self.stream_handle, device=self.kps.device).wait_event(ev)

    def extracted_event(self):
        """Event recorded on the extraction stream after the last tracked frame's extraction +
        stereo (pipelined trackers only)."""
        return self._ev_extracted[self.slot]

    def results(self):
        """Synchronise and read the frame's tracking outcome: ok follows the reference's return
        values (search >= 20, nmatchesMap >= 10, mnMatchesInliers >= 30); when a stage fails
        the later outputs are unspecified (the reference stops there)."""
        from .types import POSE_FRAME_DTYPE
        self.synchronize()
        c = self.tcounts.cpu().numpy()
        recs = self.recs.cpu().numpy().copy().view(POSE_FRAME_DTYPE).reshape(2)
        ok = c[0] >= 20 and c[2] >= 10 and c[3] >= 30
        return {"ok": bool(ok), "search_matches": int(c[0]), "outliers_mm": int(c[1]), "nmatches_map": int(c[2]),
                "inliers": int(c[3]), "outliers": int(c[4]), "tcw_mm": recs[0]["tcw"].reshape(4, 4).copy(),
                "tcw": recs[1]["tcw"].reshape(4, 4).copy(), "recs": recs}

    def synchronize(self):
        check("orbmi_extractor_synchronize", lib().orbmi_extractor_synchronize(self.extractor.handle))
        if self.pipelined:
            self._T.synchronize()

    def close(self):
        self.pose.close()
        self.matcher.close()
        self.extractor.close()


class KeyFrameData:
    """One keyframe as LocalMapping's operators read it: device-resident keypoints (cv::KeyPoint
    layout), descriptors and u_right for the GPU searches, host copies (keys, u_right, depth,
    Tcw) for the host geometry of CreateNewMapPoints, has_mp (GetMapPoint(i) != NULL, device),
    and, for a neighbour, its FeatureVector (host CSR)."""

    def __init__(self, cam, scale_factors, level_sigma2, n, d_keys, d_desc, d_ur, d_has_mp, keys, ur, depth, tcw,
                 fv=None):
        from .types import TriKeyFrame
        self.n = int(n)
        self.tcw = np.ascontiguousarray(tcw, np.float32).reshape(4, 4)
        self.keys = np.ascontiguousarray(keys)
        self.ur = np.ascontiguousarray(ur, np.float32)
        self.depth = np.ascontiguousarray(depth, np.float32)
        self.d_has_mp = d_has_mp
        self.fv = fv
        self.sf = np.ascontiguousarray(scale_factors, np.float32)
        self.sig2 = np.ascontiguousarray(level_sigma2, np.float32)
        self.view = frame_view(self.n, d_keys, d_ur, d_desc, self.tcw, cam, self.sf, cam.width, cam.height)
        mb = np.float32(np.float32(cam.bf) / np.float32(cam.fx))
        self.tri = TriKeyFrame(self.tcw.ctypes.data, self.keys.ctypes.data, self.ur.ctypes.data, self.depth.ctypes.data,
                               cam.fx, cam.fy, cam.cx, cam.cy, cam.bf, mb, self.sig2.ctypes.data, self.sf.ctypes.data)
        # HBM copies for orbmi_create_new_map_points: mvDepth and the stereo-parallax table
        import torch
        cos = np.zeros(max(self.n, 1), np.float32)
        check("orbmi_stereo_parallax_cos", lib().orbmi_stereo_parallax_cos(C.c_float(mb), self.depth.ctypes.data, self.n,
                                                                         cos.ctypes.data))
        dev = torch.device("cuda", torch.cuda.current_device())
        self.d_depth = torch.from_numpy(np.ascontiguousarray(np.resize(self.depth, max(self.n, 1)))).to(dev)
        self.d_cos = torch.from_numpy(cos).to(dev)
        self.tri_dev = TriKeyFrame(self.tcw.ctypes.data, None, None, self.d_depth.data_ptr(), cam.fx, cam.fy, cam.cx,
                                   cam.cy, cam.bf, mb, self.sig2.ctypes.data, self.sf.ctypes.data)
        # the FeatureVector in HBM too (a keyframe's is computed there by its ComputeBoW and stays)
        self.fv_dev = None
        if fv is not None:
            from .types import FeatureVectorView
            self._fv_t = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in
                          (fv.node_id.view(np.int32), fv.off, np.resize(fv.feat, max(len(fv.feat), 1)))]
            self.fv_dev = FeatureVectorView(len(fv.node_id), *[t.data_ptr() for t in self._fv_t])


class LocalMappingJob:
    """The inputs of one LocalMapping::Run iteration (src/LocalMapping.cc:47-128) for a new
    keyframe: the keyframe (its descriptors for ComputeBoW), its covisible neighbours with their
    FeatureVectors and F12 (CreateNewMapPoints / SearchInNeighbors targets), the keyframe's map
    points and the targets' map points (orbmi_mappoint records, device) for the two Fuse
    directions, the observation descriptors of the keyframe's map points for
    ComputeDistinctiveDescriptors (device CSR), and the LocalBundleAdjustment problem."""

    def __init__(self, kf, d_desc, neighbours, kf_points, target_points, obs, problem):
        self.kf, self.d_desc, self.neighbours = kf, d_desc, neighbours
        self.kf_points, self.target_points = kf_points, target_points  # (device address, count) each
        self.obs = obs                                      # (d_obs_desc, d_obs_off, n_points)
        self.problem = problem
        self.F12 = []
        for nb in neighbours:  # LocalMapping::ComputeF12 (src/LocalMapping.cc:676-693), host
            F = np.zeros(9, np.float32)
            check("orbmi_compute_f12", lib().orbmi_compute_f12(C.addressof(kf.tri), C.addressof(nb.tri), F.ctypes.data))
            self.F12.append(F)
        # the neighbours as the C ABI takes them (views of their HBM arrays)
        from .types import FeatureVectorView, TriKeyFrame
        nnb = len(neighbours)
        self.c_kf2 = (FrameView * max(nnb, 1))(*[nb.view for nb in neighbours])
        self.c_tri2 = (TriKeyFrame * max(nnb, 1))(*[nb.tri_dev for nb in neighbours])
        self.c_cos2 = (C.c_void_p * max(nnb, 1))(*[nb.d_cos.data_ptr() for nb in neighbours])
        self.c_mp2 = (C.c_void_p * max(nnb, 1))(*[nb.d_has_mp for nb in neighbours])
        self.c_fv2 = (FeatureVectorView * max(nnb, 1))(*[nb.fv_dev if nb.fv_dev is not None else nb.fv.view()
                                                          for nb in neighbours])
        self.c_F12 = np.ascontiguousarray(np.concatenate(self.F12) if nnb else np.zeros(9), np.float32)


class ChainStats(dict):
    """run_job's counts: the cheap ones at once, the search statistics (which need a device
    reduction and a read-back) on first access or materialize()."""

    _LAZY = ("triangulation_pairs", "new_points", "fuse_candidates")

    def __init__(self, lazy, **kw):
        super().__init__(**kw)
        self._lazy = lazy

    def materialize(self):
        if self._lazy is not None:
            f, self._lazy = self._lazy, None
            self.update(f())
        return self

    def __missing__(self, k):
        if k in self._LAZY and self._lazy is not None:
            return self.materialize()[k]
        raise KeyError(k)


LM_RESERVE_CUS = 0  # CUs the LocalMapping chain's stream leaves free (ORBMI_LM_RESERVE_CUS overrides)


class LocalMapper:
    """LocalMapping thread (src/LocalMapping.cc:47-128), concurrent with tracking as in the
    reference.  For every queued keyframe, in the reference's order, on the mapper's own GPU
    streams:
      ProcessNewKeyFrame    KeyFrame::ComputeBoW (DBoW2 transform) and
                            MapPoint::ComputeDistinctiveDescriptors of the keyframe's points
                            (:135-198)
      CreateNewMapPoints    SearchForTriangulation(0.6, no orientation check) against every
                            neighbour with its F12 and the triangulation / acceptance geometry,
                            pair by pair on the device (orbmi_create_new_map_points, :290-577)
      SearchInNeighbors     Fuse(neighbour, keyframe's points) for every target, Fuse(keyframe,
                            targets' points), ComputeDistinctiveDescriptors again (:589-674)
      LocalBundleAdjustment (:89-90)
    The map updates of the replayed keyframes (new points, fusions) are not applied: each job is
    self-contained, like the LocalBA problem it carries.  A job given as (problem, kf_desc) runs
    only ComputeBoW + LocalBA (the round-2 chain)."""

    def __init__(self, device=0, vocabulary=None, max_features=8192, prebow=None):
        import torch
        from .matcher import ORBmatcher
        from .optimizer import LocalBA
        self.device = device
        self.ba = LocalBA(device)
        self.matcher = ORBmatcher(device=device)
        # LocalMapping's stream kept off a few CUs, so Tracking's one-workgroup kernels always find
        # room beside a chain that fills the device (orbmi_matcher_reserve_cus)
        reserve = int(os.environ.get("ORBMI_LM_RESERVE_CUS", str(LM_RESERVE_CUS)))
        if reserve > 0:
            check("orbmi_matcher_reserve_cus", lib().orbmi_matcher_reserve_cus(self.matcher._h, reserve))
        self.voc = vocabulary  # ORBVocabulary (device handle) or None
        dev = torch.device("cuda", device)
        cap = max_features
        self.cap = cap
        self._dev = dev
        self._bufs = {}
        self._out = None
        ms = _vp()
        check("orbmi_matcher_get_stream", lib().orbmi_matcher_get_stream(self.matcher._h, C.byref(ms)))
        self._ms = torch.cuda.ExternalStream(ms.value, device=dev)  # the mapper's search stream
        # device buffers the chain writes are allocated on the stream that uses them, so the
        # caching allocator hands a freed block back only in that stream's order
        # ComputeBoW ahead (ORBMI_LM_PREBOW, default on): the next queued keyframe's transform runs
        # on the vocabulary's own stream while this keyframe's LocalBA runs on the mapper's.  It is
        # a pure function of the keyframe's descriptors (KeyFrame::ComputeBoW computes only an empty
        # mBowVec, src/KeyFrame.cc:59-70, as the KeyFrame copies a Frame's computed one), so only
        # the time it runs changes; two BowVector / FeatureVector sets alternate between the
        # keyframe in flight and the next
        if prebow is None:
            prebow = os.environ.get("ORBMI_LM_PREBOW", "1") == "1"
        self._prebow = vocabulary is not None and bool(prebow)
        with torch.cuda.stream(self._ms):
            if vocabulary is not None:  # mBowVec / mFeatVec of the keyframe, device-resident
                self.bows = [dict(word=torch.zeros(cap, dtype=torch.int32, device=dev),
                                  value=torch.zeros(cap, dtype=torch.float64, device=dev),
                                  node=torch.zeros(cap, dtype=torch.int32, device=dev),
                                  off=torch.zeros(cap + 1, dtype=torch.int32, device=dev),
                                  feat=torch.zeros(cap, dtype=torch.int32, device=dev),
                                  counts=torch.zeros(2, dtype=torch.int32, device=dev))
                             for _ in range(2 if self._prebow else 1)]
                self.bow = self.bows[0]
        self._ms.synchronize()
        # the BowVector / FeatureVector sizes, copied to pinned host words behind the transform:
        # hipHostMalloc memory, never a torch pinned tensor (_hip.py: torch would record events on
        # this library-owned stream when such a tensor is freed, after close() destroyed it)
        self._counts_hs = [PinnedWords(2) for _ in range(2 if self._prebow else 1)]
        self._counts_h = self._counts_hs[0]
        self._slot = 0
        self.bow_ahead = 0  # transforms issued beside the previous keyframe's LocalBA
        # the chain's searches and LocalBA are in order on one stream, so that the process's
        # streams stay within the device's hardware queues (orbmi_ba_set_stream); without the
        # transform ahead, ComputeBoW joins them there
        self._one_stream = os.environ.get("ORBMI_LM_STREAMS", "one") == "one"
        if self._one_stream:
            check("orbmi_ba_set_stream", lib().orbmi_ba_set_stream(self.ba._h, ms))
            if vocabulary is not None and not self._prebow:
                check("orbmi_vocabulary_set_stream", lib().orbmi_vocabulary_set_stream(vocabulary._h, ms))
        self._vs = None
        self._hook_cb = None
        self._job_start_ev = None
        self._cur_job = None
        if self._prebow:
            vs = _vp()
            check("orbmi_vocabulary_get_stream", lib().orbmi_vocabulary_get_stream(vocabulary._h, C.byref(vs)))
            self._vs = torch.cuda.ExternalStream(vs.value, device=dev)
            # the next keyframe's transform is issued from LocalBA's enqueued hook: after the solve's
            # work is on the stream and before the host waits for it, so the host's issue time is
            # off the chain and the transform runs beside the one-workgroup solve
            self._hook_cb = C.CFUNCTYPE(None, C.c_void_p)(self._on_ba_enqueued)
            check("orbmi_ba_set_enqueued_hook", lib().orbmi_ba_set_enqueued_hook(
                self.ba._h, C.cast(self._hook_cb, C.c_void_p), None))
        self.q: queue.Queue = queue.Queue()
        self.job_events = None  # a list: per job (start event, end event, host start, host end)
        self.done = 0
        self.last = None
        self.last_chain = None
        self.error = None
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _buf(self, name, shape, dtype):
        import torch
        b = self._bufs.get(name)
        if b is None or b.numel() < int(np.prod(shape)) or b.dtype != dtype:
            with torch.cuda.stream(self._ms):  # allocated on the stream that writes it
                b = torch.empty(int(np.prod(shape)), dtype=dtype, device=self._dev)
            self._bufs[name] = b
        return b

    def _run(self):
        while True:
            job = self.q.get()
            if job is None:
                self.q.task_done()
                return
            try:
                if isinstance(job, LocalMappingJob):
                    self.last_chain = self.run_job(job)
                else:
                    self._bow_and_ba(*job)
                self.done += 1
            except Exception as e:  # surfaced by wait()
                self.error = e
            self.q.task_done()

    def _bow_and_ba(self, problem, kf_desc):
        if self.voc is not None and kf_desc is not None:
            d_desc, n = kf_desc
            b = self.bow
            self.voc.transform_device(d_desc, n, None, 4, b["word"].data_ptr(), b["value"].data_ptr(),
                                      b["node"].data_ptr(), b["off"].data_ptr(), b["feat"].data_ptr(),
                                      b["counts"].data_ptr())
            bow_done = self._bow_event()
        # LocalBundleAdjustment reads poses, points and observations, never the BowVector (they run
        # in order on the mapper's stream, or side by side with the transform ahead)
        self.last = self.ba.run(problem)
        if self.voc is not None and kf_desc is not None:
            bow_done.synchronize()

    def run_job(self, job: LocalMappingJob):
        """One LocalMapping::Run iteration (see the class doc) -> counts of what it found.  The
        chain runs in order on the mapper's stream with one host synchronisation before
        CreateNewMapPoints (the FeatureVector's node count sizes its search) and the one LocalBA
        ends with; the statistics of the searches are read lazily (ChainStats)."""
        import torch
        from .types import FeatureVector, FeatureVectorView
        L = lib()
        m = self.matcher._h
        kf = job.kf
        je = self.job_events  # diagnostics (bench --frame-events): the job's span on the stream
        if je is not None:
            t_host0 = time.perf_counter()
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(self._ms)
            marks = []

        def mark(name):  # a stage boundary on the mapper's stream (diagnostics only)
            if je is not None:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(self._ms)
                marks.append((name, ev))
        # ---- ProcessNewKeyFrame: ComputeBoW (transform of the keyframe's descriptors) and the
        # ComputeDistinctiveDescriptors of the keyframe's map points
        if self._prebow:  # issued ahead while the previous keyframe's LocalBA ran, or now
            self._job_start_ev = torch.cuda.Event()
            self._job_start_ev.record(self._ms)  # the previous keyframes' work: a free set's last reader
            self._cur_job = job
            slot, _ = job._bow if getattr(job, "_bow", None) is not None else self._issue_bow(job)
            job._bow = None
            b, counts_h = self.bows[slot], self._counts_hs[slot]
            self.bow = b
        else:  # enqueued back to back with ComputeDistinctiveDescriptors
            b, counts_h = self.bow, self._counts_h
            self.voc.transform_device(job.d_desc, kf.n, None, 4, b["word"].data_ptr(), b["value"].data_ptr(),
                                      b["node"].data_ptr(), b["off"].data_ptr(), b["feat"].data_ptr(),
                                      b["counts"].data_ptr())
            if not self._one_stream:  # the transform ran on the vocabulary's own stream
                self.voc.synchronize()
            # mBowVec / mFeatVec sizes, behind the transform on the mapper's stream
            counts_h.copy_async(b["counts"].data_ptr(), self._ms.cuda_stream)
        d_obs, d_off, npts = job.obs
        best = self._buf("best", (max(npts, 1),), torch.int32)
        dsc = self._buf("dsc", (max(npts, 1) * 32,), torch.uint8)

        def distinctive():
            check("orbmi_compute_distinctive_descriptors", L.orbmi_compute_distinctive_descriptors(
                m, _vp(d_obs), _vp(d_off), int(npts), _vp(best.data_ptr()), _vp(dsc.data_ptr())))
        # enqueued first, so the stream is busy while the host prepares CreateNewMapPoints (putting
        # CreateNewMapPoints first left the stream idle for that setup: 2,836-2,881 against
        # 2,914-2,949 frames/s, profiles/r06/lm_prebow_ab.txt)
        distinctive()
        # the later stages' buffers, prepared while the GPU runs the calls above
        nnb = len(job.neighbours)
        tri = self._buf("tri", (max(nnb, 1) * kf.n,), torch.int32)
        tri_ok = self._buf("tri_ok", (max(nnb, 1) * kf.n,), torch.uint8)
        x3d = self._buf("tri_x3d", (max(nnb, 1) * kf.n * 3,), torch.float32)
        d_kp, n_kp = job.kf_points
        d_tp, n_tp = job.target_points
        bi = self._buf("fuse_bi", (max(nnb * n_kp + n_tp, 1),), torch.int32)
        bd = self._buf("fuse_bd", (max(nnb * n_kp + n_tp, 1),), torch.int32)
        kf2 = job.c_kf2
        mark("bow_distinctive")
        # waits for the size copy only (whatever the stream mode).  With the transform ahead the
        # copy follows the transform on the vocabulary's stream, so once the host has read the
        # sizes the FeatureVector is complete too and the mapper's stream needs no cross-stream
        # wait (a wait packet costs the stream ~10 us)
        nw, nn = counts_h.read()
        # ---- CreateNewMapPoints: every neighbour's SearchForTriangulation and the triangulation /
        # acceptance geometry on the device, in the reference's pair order (orbmi_create_new_map_points)
        fv1 = FeatureVectorView(nn, b["node"].data_ptr(), b["off"].data_ptr(), b["feat"].data_ptr())
        if nnb:
            check("orbmi_create_new_map_points", L.orbmi_create_new_map_points(
                m, C.addressof(kf.view), C.addressof(kf.tri_dev), _vp(kf.d_cos.data_ptr()), _vp(kf.d_has_mp),
                C.addressof(fv1), nnb, kf2, job.c_tri2, job.c_cos2, job.c_mp2, job.c_fv2, job.c_F12.ctypes.data,
                _vp(tri.data_ptr()), _vp(tri_ok.data_ptr()), _vp(x3d.data_ptr())))
        nt = nnb * kf.n
        mark("create_new_map_points")
        # ---- SearchInNeighbors: Fuse(target, keyframe's points) per target, Fuse(keyframe, targets' points)
        if nnb:
            check("orbmi_fuse_search_batch", L.orbmi_fuse_search_batch(
                m, nnb, kf2, _vp(d_kp), None, int(n_kp), 3.0, _vp(bi.data_ptr()), _vp(bd.data_ptr()), None))
        o = nnb * n_kp
        check("orbmi_fuse_search", L.orbmi_fuse_search(
            m, C.addressof(kf.view), _vp(d_tp), None, int(n_tp), 3.0, _vp(bi.data_ptr() + 4 * o),
            _vp(bd.data_ptr() + 4 * o), None))
        mark("fuse")
        # ComputeDistinctiveDescriptors + UpdateNormalAndDepth of the keyframe's points after fusion
        check("orbmi_compute_distinctive_descriptors", L.orbmi_compute_distinctive_descriptors(
            m, _vp(d_obs), _vp(d_off), int(npts), _vp(best.data_ptr()), _vp(dsc.data_ptr())))
        mark("distinctive")
        # (the next queued keyframe's ComputeBoW: _on_ba_enqueued, from inside this call)
        # ---- LocalBundleAdjustment (same stream, so it runs behind the searches above)
        self.last = self.ba.run(job.problem)
        ms = self._ms
        if je is not None:  # LocalBA returned: its work is complete
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(ms)
            je.append((e0, e1, t_host0, time.perf_counter(), marks))

        def stats():  # what the searches found (statistics only: off the chain's path)
            ms.synchronize()
            c = torch.stack([(tri[:nt] >= 0).sum(), tri_ok[:nt].sum(dtype=torch.int64),
                             (bi[:o + n_tp] >= 0).sum()]).cpu().numpy()
            return {"triangulation_pairs": int(c[0]), "new_points": int(c[1]), "fuse_candidates": int(c[2])}
        out = ChainStats(stats, bow_words=nw, local_ba_iterations=list(self.last["iterations"]))
        self._out = dict(tri=lambda: tri[:nt].cpu().numpy().reshape(nnb, kf.n),
                         tri_ok=lambda: tri_ok[:nt].cpu().numpy().reshape(nnb, kf.n),
                         x3d=lambda: x3d[:3 * nt].cpu().numpy().reshape(nnb, kf.n, 3),
                         best=best, dsc=dsc, bi=bi, bd=bd, n_fuse=o + n_tp,
                         fv=lambda: FeatureVector.from_csr(b["node"][:nn].cpu().numpy().view(np.uint32),
                                                           b["off"][:nn + 1].cpu().numpy(),
                                                           b["feat"][:kf.n].cpu().numpy()))
        return out

    def _on_ba_enqueued(self, _arg):
        """LocalBA's enqueued hook (orbmi_ba_set_enqueued_hook): the next queued keyframe's
        ComputeBoW, beside the solve.  Never raises into the C caller (errors surface in wait())."""
        try:
            with self.q.mutex:
                nxt = self.q.queue[0] if self.q.queue else None
            if isinstance(nxt, LocalMappingJob) and nxt is not self._cur_job and getattr(nxt, "_bow", None) is None:
                self._issue_bow(nxt, after=self._job_start_ev)
                self.bow_ahead += 1
        except Exception as e:  # pragma: no cover
            self.error = e

    def _issue_bow(self, job, after=None):
        """ComputeBoW of job's keyframe on the vocabulary's stream into the next BowVector /
        FeatureVector set (the other one belongs to the keyframe in flight), its sizes to that
        set's pinned words; -> (set, event).  The transform waits for `after` (an event on the
        mapper's stream behind the set's previous reader), else for everything enqueued there."""
        import torch
        slot = self._slot
        self._slot = (slot + 1) % len(self.bows)
        b = self.bows[slot]
        if after is None:  # behind everything enqueued on the mapper's stream so far
            after = torch.cuda.Event()
            after.record(self._ms)
        self._vs.wait_event(after)
        self.voc.transform_device(job.d_desc, job.kf.n, None, 4, b["word"].data_ptr(), b["value"].data_ptr(),
                                  b["node"].data_ptr(), b["off"].data_ptr(), b["feat"].data_ptr(), b["counts"].data_ptr())
        self._counts_hs[slot].copy_async(b["counts"].data_ptr(), self._vs.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(self._vs)
        job._bow = (slot, ev)
        return job._bow

    def _bow_event(self):
        """Event recorded on the vocabulary's stream after the transform just enqueued."""
        import torch
        s = C.c_void_p()
        check("orbmi_vocabulary_get_stream", lib().orbmi_vocabulary_get_stream(self.voc._h, C.byref(s)))
        ev = torch.cuda.Event()
        ev.record(torch.cuda.ExternalStream(s.value, device=torch.device("cuda", self.device)))
        return ev

    def insert_keyframe(self, problem_or_job, kf_desc=None):
        """Queue a keyframe: a LocalMappingJob (the whole LocalMapping chain), or (LocalBA
        problem, (device address of its n x 32 descriptors, n)) for ComputeBoW + LocalBA only."""
        if isinstance(problem_or_job, LocalMappingJob):
            self.q.put(problem_or_job)
        else:
            self.q.put((problem_or_job, kf_desc))

    def wait(self):
        self.q.join()
        if self.error is not None:
            raise self.error

    def close(self):
        """Stop the thread, drain the mapper's stream, settle everything that refers to it (the
        lazy statistics, the result views, the buffers, the pinned words), then destroy the
        handles that own the stream.  Nothing used on the stream outlives it."""
        self.q.put(None)
        self.t.join()
        self._ms.synchronize()
        if isinstance(self.last_chain, ChainStats):
            self.last_chain.materialize()  # its closure synchronises self._ms
        self._out = None
        self._bufs = {}
        if getattr(self, "_hook_cb", None) is not None and getattr(self.ba, "_h", None):
            check("orbmi_ba_set_enqueued_hook", lib().orbmi_ba_set_enqueued_hook(self.ba._h, None, None))
        if self._vs is not None:
            self._vs.synchronize()
        for c in self._counts_hs:
            c.close()
        if self._one_stream and self.voc is not None and getattr(self.voc, "_h", None):  # it outlives the mapper
            check("orbmi_vocabulary_set_stream", lib().orbmi_vocabulary_set_stream(self.voc._h, None))
        self.ba.close()
        self.matcher.close()


def gather_stream_features(dist, desc, kps, count):
    """Config 4 exchange: all-gather every stream's left descriptors (cap x 32 u8), keypoints
    (cap x 7 x i32, cv::KeyPoint layout) and count over the process group (RCCL over xGMI on
    the GPU, gloo on the CPU).  Returns (desc[W,cap,32], kps[W,cap,7], counts[W])."""
    import torch
    world = dist.get_world_size()

    def gather(t):
        t = t.contiguous()
        out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t)  # rank-major concatenation along dim 0
        return out.view((world,) + tuple(t.shape))

    g_desc, g_kps, g_cnt = gather(desc), gather(kps), gather(count)
    return g_desc, g_kps, g_cnt


def match_cross_stream(matcher_handle, q_desc, nq, nq_device, g_desc, seg_counts, skip_seg, out, th=50, ratio=0.6,
                       nmatches=None):
    """orbmi_match_descriptors_segments over the gathered segments (device tensors)."""
    world, cap = int(g_desc.shape[0]), int(g_desc.shape[1])
    check("orbmi_match_descriptors_segments", lib().orbmi_match_descriptors_segments(
        matcher_handle, _vp(q_desc), int(nq), _vp(nq_device) if nq_device else None, _vp(g_desc.data_ptr()), world, cap,
        _vp(seg_counts.data_ptr()), int(skip_seg), int(th), float(ratio), _vp(out.data_ptr()),
        C.byref(nmatches) if nmatches is not None else None))


class StreamExchange:
    """Config 4: after each tracked frame, all-gather the stream's left
    descriptors + keypoints over the process group and match them against the other streams'
    (orbmi_match_descriptors_segments; build-defined cross-stream matching, no reference
    counterpart).  The exchange runs on its own stream X (a second matcher handle's): it waits
    only for the frame's extraction event, so tracking on T never waits for the collective, and
    the frame's slot is held until X has read it (StereoTracker.hold_slot), so the extraction
    two frames later cannot overwrite features the gather or the match still reads."""

    def __init__(self, tracker, dist, device=0):
        import torch
        from .matcher import ORBmatcher
        self.tr, self.dist = tracker, dist
        self.matcher = ORBmatcher(device=device)
        x = _vp()
        check("orbmi_matcher_get_stream", lib().orbmi_matcher_get_stream(self.matcher._h, C.byref(x)))
        self.X = torch.cuda.ExternalStream(x.value, device=torch.device("cuda", device))
        self.xmatch = torch.full((tracker.cap,), -1, dtype=torch.int32, device=torch.device("cuda", device))
        self._keep = None

    def exchange(self):
        """Enqueue the exchange of the frame tracker.track() enqueued last."""
        import torch
        tr = self.tr
        if tr.pipelined:
            self.X.wait_event(tr.extracted_event())
        else:
            self.X.wait_stream(torch.cuda.ExternalStream(tr.stream_handle, device=tr.kps.device))
        with torch.cuda.stream(self.X):
            g_desc, g_kps, g_cnt = gather_stream_features(self.dist, tr.desc[0], tr.kps[0], tr.counts[:1])
        match_cross_stream(self.matcher._h, tr.desc.data_ptr(), tr.cap, tr.counts.data_ptr(), g_desc,
                           g_cnt.view(-1), self.dist.get_rank(), self.xmatch)
        tr.hold_slot(self.X)
        self._keep = (g_desc, g_kps, g_cnt)  # alive until X has consumed them (next exchange)
        return self._keep

    def synchronize(self):
        self.X.synchronize()

    def close(self):
        self.matcher.close()
