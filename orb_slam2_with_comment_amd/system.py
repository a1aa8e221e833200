"""Stereo SLAM host integration: System::TrackStereo, the stereo
Tracking state machine and a synchronous LocalMapping, driving the MI355X operators.

This module is the host code around the GPU path, in the reference's own structure:

  System::TrackStereo        -> StereoSLAM.TrackStereo              src/System.cc:110-159
  Tracking::Track (stereo)   -> StereoSLAM._track                   src/Tracking.cc:287-581
  StereoInitialization       -> StereoSLAM._stereo_initialization   src/Tracking.cc:584-636
  TrackReferenceKeyFrame     -> StereoSLAM._track_reference_kf      src/Tracking.cc:871-917
  TrackWithMotionModel       -> StereoSLAM._track_motion_model      src/Tracking.cc:997-1063
  TrackLocalMap              -> StereoSLAM._track_local_map         src/Tracking.cc:1075-1104
  UpdateLocalKeyFrames/Points, SearchLocalPoints                    src/Tracking.cc:1345-1580
  NeedNewKeyFrame / CreateNewKeyFrame                               src/Tracking.cc:1140-1330
  LocalMapping::ProcessNewKeyFrame + LocalBundleAdjustment          src/LocalMapping.cc:152-200, :89-90
  KeyFrame::UpdateConnections / MapPoint bookkeeping                src/KeyFrame.cc, src/MapPoint.cc
  System::SaveTrajectoryKITTI / SaveTrajectoryTUM / SaveKeyFrameTrajectoryTUM
                                                                    src/System.cc:334-486

Every per-keypoint operation (ORBextractor, ComputeStereoMatches, ComputeBoW, the three
SearchBy* matchers, PoseOptimization, ComputeDistinctiveDescriptors, LocalBundleAdjustment)
goes through a *backend*; the product backend is `GpuBackend` (liborbmi.so on MI355X, no CPU
fallback: a missing library raises).  The host logic here only keeps the map and the
reference's bookkeeping.  Tests drive the same host logic with an oracle-backed backend
(tests/slam_backends.py) to prove that the GPU run yields the oracle's trajectory.

Deterministic replacements of the reference's unordered behaviour (documented in DESIGN.md §9):
  * LocalMapping runs synchronously after each new keyframe (the reference runs it on its own
    thread; with LocalMapping always idle NeedNewKeyFrame's c1b holds, as on a fast machine).
  * std::map<KeyFrame*, ...> iteration (pointer order) is keyframe-id order; covisibility ties
    sort by id like ascending heap addresses do.
  * Relocalisation and loop closing are not part of this path (out of scope).
  * ORBmatcher::Fuse searches all of a call's points on the backend at once, then replays the
    map updates in list order (re-checking isBad / IsInKeyFrame); descriptors of points that
    gained observations by MapPoint::Replace are recomputed before the next Fuse call.
"""
from __future__ import annotations

import dataclasses

import numpy as np

from .types import (LF_HAS_MP, LF_OUTLIER, LFPOINT_DTYPE, MAPPOINT_DTYPE, MP_BAD, MP_HAS_OBS, MP_SEEN,
                    FeatureVector, Frame)

NO_IMAGES_YET, NOT_INITIALIZED, OK, LOST = 0, 1, 2, 3   # Tracking::eTrackingState (include/Tracking.h)

# Where a thread resumes after releasing the map lock (include/orbmi_debug.h ORBMI_SCHED_*): the
# generators below yield these at the points where the native loop (csrc/slam.cpp) releases
# its map lock around a GPU call, so a recorded concurrent schedule can be replayed here
T_FRAME, T_BOW, T_POSE, T_LF, T_LOCAL, T_RESET = 1, 2, 3, 4, 5, 6
L_JOB, L_DISTINCTIVE, L_CREATE, L_CREATE_PAIR, L_FUSE_BATCH, L_FUSE_REFRESH, L_FUSE, L_BA, L_BOW = range(16, 25)


KF_STATE_PROCESS, KF_STATE_CREATE, KF_STATE_FUSE = 0, 1, 2   # ORBMI_KF_STATE_* (include/orbmi_debug.h)
FNV0 = 2166136261


def _fnv(h: int, words) -> int:
    """h = (h ^ w) * 16777619 mod 2^32 over 32-bit words (the native state record's hash)."""
    for w in np.asarray(words).astype(np.int64).tolist():
        h = ((h ^ (w & 0xFFFFFFFF)) * 16777619) & 0xFFFFFFFF
    return h


def _slot_hash(kf) -> int:
    return _fnv(FNV0, [-1 if mp is None else mp.id for mp in kf.map_points])


def _i32(v: int) -> int:
    v = int(v) & 0xFFFFFFFF
    return v - (1 << 32) if v >= 1 << 31 else v


class ScheduleMismatch(RuntimeError):
    """A recorded concurrent schedule does not fit this host logic (replay_schedule)."""


# ---- float32 pose algebra (cv::Mat CV_32F products accumulate in double, src/Converter.cc) --
def _mul(*ms) -> np.ndarray:
    out = np.asarray(ms[0], np.float32)
    for m in ms[1:]:
        out = (out.astype(np.float64) @ np.asarray(m, np.float32).astype(np.float64)).astype(np.float32)
    return out


def pose_inverse(T: np.ndarray) -> np.ndarray:
    """Twc from Tcw as Frame::UpdatePoseMatrices does: Rwc = Rcw^T, Ow = -Rcw^T tcw."""
    T = np.asarray(T, np.float32)
    Rwc = T[:3, :3].T.copy()
    out = np.eye(4, dtype=np.float32)
    out[:3, :3] = Rwc
    out[:3, 3] = -_mul(Rwc, T[:3, 3:4])[:, 0]
    return out


def quaternion_xyzw(R) -> np.ndarray:
    """Converter::toQuaternion (src/Converter.cc:137-149): Eigen::Quaterniond(Matrix3d) of a
    float rotation, returned as float [x, y, z, w]."""
    m = np.asarray(R, np.float32).astype(np.float64)
    q = np.zeros(4)  # x y z w
    t = m[0, 0] + m[1, 1] + m[2, 2]
    if t > 0:
        t = np.sqrt(t + 1.0)
        q[3] = 0.5 * t
        t = 0.5 / t
        q[0], q[1], q[2] = (m[2, 1] - m[1, 2]) * t, (m[0, 2] - m[2, 0]) * t, (m[1, 0] - m[0, 1]) * t
    else:
        i = 1 if m[1, 1] > m[0, 0] else 0
        if m[2, 2] > m[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = np.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
        q[i] = 0.5 * t
        t = 0.5 / t
        q[3] = (m[k, j] - m[j, k]) * t
        q[j] = (m[j, i] + m[i, j]) * t
        q[k] = (m[k, i] + m[i, k]) * t
    return q.astype(np.float32)


# ---- map model (src/KeyFrame.cc, src/MapPoint.cc) ------------------------------------------
@dataclasses.dataclass(eq=False, repr=False)
class KeyFrame:
    """The fields of ORB_SLAM2::KeyFrame this path reads; also the graph node type of
    optimizer.gather_local_ba (id, tcw, keys_un, u_right, inv_level_sigma2, cam, map_points,
    covisible, bad)."""
    id: int
    frame_id: int
    timestamp: float
    tcw: np.ndarray
    keys_un: np.ndarray
    desc: np.ndarray
    u_right: np.ndarray
    depth: np.ndarray
    inv_level_sigma2: np.ndarray
    scale_factors: np.ndarray
    cam: object
    map_points: list
    feat_vec: object = None
    covisible: list = dataclasses.field(default_factory=list)  # mvpOrderedConnectedKeyFrames
    conn: dict = dataclasses.field(default_factory=dict)       # mConnectedKeyFrameWeights
    parent: object = None
    children: list = dataclasses.field(default_factory=list)  # mspChildrens (iterated in id order)
    first_connection: bool = True
    bad: bool = False
    fuse_target_for_kf: int = -1    # mnFuseTargetForKF
    tcp: np.ndarray = None          # mTcp (set when the keyframe turns bad)

    @property
    def Ow(self) -> np.ndarray:
        """Camera centre, cached per pose array (poses are replaced, never edited in place)."""
        c = self.__dict__.get("_ow")
        if c is None or c[0] is not self.tcw:
            c = (self.tcw, pose_inverse(self.tcw)[:3, 3].copy())
            self.__dict__["_ow"] = c
        return c[1]

    def tracked_map_points(self, min_obs: int) -> int:
        """KeyFrame::TrackedMapPoints (src/KeyFrame.cc:166-193)."""
        n = 0
        for mp in self.map_points:
            if mp is not None and not mp.bad and (min_obs <= 0 or mp.nobs >= min_obs):
                n += 1
        return n

    def add_connection(self, kf, weight):
        """KeyFrame::AddConnection + UpdateBestCovisibles (src/KeyFrame.cc:97-135): the ordered
        list holds every connection, heaviest first."""
        self.conn[kf] = weight
        self.covisible = [k for w, _, k in sorted(((w, k.id, k) for k, w in self.conn.items()),
                                                 key=lambda p: (p[0], p[1]), reverse=True)]

    def best_covisibility(self, n: int) -> list:
        return self.covisible[:n]

    def get_weight(self, kf) -> int:
        return self.conn.get(kf, 0)

    def erase_connection(self, kf):
        """KeyFrame::EraseConnection + UpdateBestCovisibles (src/KeyFrame.cc:567-581)."""
        if kf in self.conn:
            del self.conn[kf]
            self.covisible = [k for w, _, k in sorted(((w, k.id, k) for k, w in self.conn.items()),
                                                     key=lambda p: (p[0], p[1]), reverse=True)]

    def change_parent(self, kf):
        """KeyFrame::ChangeParent (src/KeyFrame.cc): mpParent = pKF; pKF->AddChild(this)."""
        self.parent = kf
        if self not in kf.children:
            kf.children.append(self)

    def set_bad(self):
        """KeyFrame::SetBadFlag (src/KeyFrame.cc:467-559): drop the covisibility links and the
        observations, hand the children to the best-connected parent candidates (spanning
        tree), keep Tcp for the trajectory.  std::set / std::map pointer order -> id order."""
        if self.id == 0:
            return
        for kf in sorted(self.conn, key=lambda k: k.id):
            kf.erase_connection(self)
        for mp in self.map_points:
            if mp is not None:
                mp.erase_observation(self)
        self.conn = {}
        self.covisible = []
        candidates = {self.parent}
        children = sorted(self.children, key=lambda k: k.id)
        while children:
            cont, best, pc, pp = False, -1, None, None
            for kf in children:
                if kf.bad:
                    continue
                for c in kf.covisible:
                    for cand in sorted(candidates, key=lambda k: k.id):
                        if c.id == cand.id:
                            w = kf.get_weight(c)
                            if w > best:
                                pc, pp, best, cont = kf, c, w, True
            if not cont:
                break
            pc.change_parent(pp)
            candidates.add(pc)
            children.remove(pc)
            self.children.remove(pc)
        for kf in children:
            kf.change_parent(self.parent)
        self.children = []
        if self in self.parent.children:
            self.parent.children.remove(self)
        self.tcp = _mul(self.tcw, pose_inverse(self.parent.tcw))
        self.bad = True

    def update_connections(self):
        """KeyFrame::UpdateConnections (src/KeyFrame.cc:285-371)."""
        counter: dict = {}
        for mp in self.map_points:
            if mp is None or mp.bad:
                continue
            for kf in mp.observations:
                if kf is not self:
                    counter[kf] = counter.get(kf, 0) + 1
        if not counter:
            return
        th = 15
        nmax, kfmax = 0, None
        pairs = []
        for kf in sorted(counter, key=lambda k: k.id):
            w = counter[kf]
            if w > nmax:
                nmax, kfmax = w, kf
            if w >= th:
                pairs.append((w, kf.id, kf))
                kf.add_connection(self, w)
        if not pairs:
            pairs.append((nmax, kfmax.id, kfmax))
            kfmax.add_connection(self, nmax)
        pairs.sort(key=lambda p: (p[0], p[1]), reverse=True)
        self.conn = counter
        self.covisible = [p[2] for p in pairs]
        if self.first_connection and self.id != 0:
            self.parent = self.covisible[0]
            self.parent.children.append(self)
            self.first_connection = False


@dataclasses.dataclass(eq=False, repr=False)
class MapPoint:
    id: int
    pos: np.ndarray                 # float32[3]
    ref_kf: KeyFrame
    desc: np.ndarray = None         # distinctive descriptor (32 B)
    normal: np.ndarray = None
    max_distance: np.float32 = np.float32(0)
    min_distance: np.float32 = np.float32(0)
    observations: dict = dataclasses.field(default_factory=dict)   # KeyFrame -> keypoint index
    nobs: int = 0
    bad: bool = False
    first_kf_id: int = 0            # mnFirstKFid
    visible: int = 1                # mnVisible
    found: int = 1                  # mnFound
    replaced: object = None         # mpReplaced
    fuse_candidate_for_kf: int = -1  # mnFuseCandidateForKF

    def found_ratio(self) -> np.float32:
        """MapPoint::GetFoundRatio: static_cast<float>(mnFound) / mnVisible."""
        return np.float32(np.float32(self.found) / np.float32(self.visible))

    def replace(self, other) -> bool:
        """MapPoint::Replace (src/MapPoint.cc:172-215): other takes over this point's
        observations (keyframe-id order); this point turns bad.  Returns True when other gained
        observations (its distinctive descriptor is then recomputed by the caller)."""
        if other.id == self.id:
            return False
        obs = sorted(self.observations.items(), key=lambda o: o[0].id)
        self.observations = {}
        self.bad = True
        self.replaced = other
        for kf, idx in obs:
            if kf not in other.observations:
                kf.map_points[idx] = other              # KeyFrame::ReplaceMapPointMatch
                other.add_observation(kf, idx)
            else:
                kf.map_points[idx] = None               # KeyFrame::EraseMapPointMatch
        other.found += self.found
        other.visible += self.visible
        return True

    def add_observation(self, kf: KeyFrame, idx: int):
        """MapPoint::AddObservation (src/MapPoint.cc:90-105): stereo observations count 2."""
        if kf in self.observations:
            return
        self.observations[kf] = idx
        self.nobs += 2 if kf.u_right[idx] >= 0 else 1

    def erase_observation(self, kf: KeyFrame):
        """MapPoint::EraseObservation (src/MapPoint.cc:111-137)."""
        if kf not in self.observations:
            return
        idx = self.observations.pop(kf)
        self.nobs -= 2 if kf.u_right[idx] >= 0 else 1
        if self.ref_kf is kf and self.observations:
            self.ref_kf = min(self.observations, key=lambda k: k.id)
        if self.nobs <= 2:
            self.set_bad()

    def set_bad(self):
        """MapPoint::SetBadFlag (src/MapPoint.cc:151-170)."""
        self.bad = True
        for kf, idx in self.observations.items():
            if kf.map_points[idx] is self:
                kf.map_points[idx] = None
        self.observations = {}

    def update_normal_and_depth(self):
        """MapPoint::UpdateNormalAndDepth (src/MapPoint.cc:339-390) in float32."""
        if self.bad or not self.observations:
            return
        normal = np.zeros(3, np.float32)
        for kf in sorted(self.observations, key=lambda k: k.id):
            v = (self.pos - kf.Ow).astype(np.float32)   # normali / cv::norm(normali): alpha in double
            normal = (normal + (v.astype(np.float64) * (1.0 / np.linalg.norm(v.astype(np.float64)))).astype(np.float32))
        PC = (self.pos - self.ref_kf.Ow).astype(np.float32)
        dist = np.float32(np.linalg.norm(PC.astype(np.float64)))
        level = int(self.ref_kf.keys_un[self.observations[self.ref_kf]]["octave"])
        sf = self.ref_kf.scale_factors
        self.max_distance = np.float32(dist * sf[level])
        self.min_distance = np.float32(self.max_distance / sf[len(sf) - 1])
        self.normal = (normal.astype(np.float64) * (1.0 / len(self.observations))).astype(np.float32)


def update_normals_and_depths(mps: list):
    """MapPoint::UpdateNormalAndDepth for many points at once, with the per-point method's exact
    float32 arithmetic and summation order (observing keyframes in id order)."""
    pts = [mp for mp in mps if not mp.bad and mp.observations]
    if not pts:
        return
    owner, cen = [], []
    for j, mp in enumerate(pts):
        for kf in sorted(mp.observations, key=lambda k: k.id):
            owner.append(j)
            cen.append(kf.Ow)
    owner = np.asarray(owner)
    pos = np.array([mp.pos for mp in pts], np.float32)
    v = (pos[owner] - np.asarray(cen, np.float32)).astype(np.float32)
    v64 = v.astype(np.float64)
    terms = (v64 * (1.0 / np.sqrt(np.sum(v64 * v64, axis=1)))[:, None]).astype(np.float32)
    normal = np.zeros((len(pts), 3), np.float32)
    np.add.at(normal, owner, terms)          # float32, sequential in observation order
    cnt = np.bincount(owner, minlength=len(pts)).astype(np.float64)
    normal = (normal.astype(np.float64) * (1.0 / cnt)[:, None]).astype(np.float32)
    ref_ow = np.array([mp.ref_kf.Ow for mp in pts], np.float32)
    PC = (pos - ref_ow).astype(np.float32).astype(np.float64)
    dist = np.sqrt(np.sum(PC * PC, axis=1)).astype(np.float32)
    for j, mp in enumerate(pts):
        sf = mp.ref_kf.scale_factors
        level = int(mp.ref_kf.keys_un[mp.observations[mp.ref_kf]]["octave"])
        mp.max_distance = np.float32(dist[j] * sf[level])
        mp.min_distance = np.float32(mp.max_distance / sf[len(sf) - 1])
        mp.normal = normal[j].copy()


# ---- the per-frame state Tracking keeps (include/Frame.h) ----------------------------------
@dataclasses.dataclass(eq=False, repr=False)
class TrackedFrame:
    id: int
    timestamp: float
    keys: np.ndarray
    desc: np.ndarray
    u_right: np.ndarray
    depth: np.ndarray
    tcw: np.ndarray = None
    map_points: list = None          # mvpMapPoints
    outlier: np.ndarray = None       # mvbOutlier
    ref_kf: KeyFrame = None
    feat_vec: object = None

    @property
    def n(self):
        return len(self.keys)


class GpuBackend:
    """The MI355X operators behind the reference's interfaces (liborbmi.so; raises when the
    library or the GPU is missing -- there is no CPU path)."""

    def __init__(self, settings, device: int = 0, vocabulary=None):
        from .matcher import ORBmatcher
        from .optimizer import LocalBA, PoseOptimizer
        from .orb import ORBextractor
        s = settings
        self.left = ORBextractor(s.n_features, float(s.scale_factor), s.n_levels, s.ini_th_fast, s.min_th_fast,
                                 device=device)
        self.right = ORBextractor(s.n_features, float(s.scale_factor), s.n_levels, s.ini_th_fast, s.min_th_fast,
                                  device=device)
        self.scale_factors = np.ascontiguousarray(self.left.GetScaleFactors(), np.float32)
        self.inv_level_sigma2 = np.ascontiguousarray(self.left.GetInverseScaleSigmaSquares(), np.float32)
        self.m_lf = ORBmatcher(0.9, True, device=device)     # src/Tracking.cc:1002
        self.m_local = ORBmatcher(0.8, True, device=device)  # src/Tracking.cc:1391
        self.m_bow = ORBmatcher(0.7, True, device=device)    # src/Tracking.cc:878
        self.m_util = ORBmatcher(device=device)
        self.m_tri = ORBmatcher(0.6, False, device=device)   # src/LocalMapping.cc:301
        self.pose = PoseOptimizer(device)
        self.ba = LocalBA(device)
        self.vocab = None
        if vocabulary is not None:
            from .vocabulary import ORBVocabulary
            self.vocab = ORBVocabulary(vocabulary, device)

    def extract_stereo(self, imL, imR):
        """Frame::Frame (stereo) (src/Frame.cc:58-100): ORBextractor on both images and
        ComputeStereoMatches -> keys, desc, mvuRight, mvDepth."""
        from .orb import compute_stereo_matches
        kl, dl = self.left(imL)
        kr, dr = self.right(imR)
        n = len(kl)
        if dl is None:
            dl = np.zeros((0, 32), np.uint8)
        u, d = compute_stereo_matches(self.left, self.right, self.cam_bf, self.cam_fx, n)
        return kl, dl, u, d

    def bind_camera(self, cam):
        self.cam_bf, self.cam_fx = float(cam.bf), float(cam.fx)

    def compute_bow(self, desc):
        if self.vocab is None:
            raise RuntimeError("TrackReferenceKeyFrame needs a vocabulary (StereoSLAM(vocabulary=...))")
        words, _, fv = self.vocab.ComputeBoW(desc)
        fv.n_words = len(words)   # (the BowVector's size, for the per-keyframe state record)
        return fv

    def search_by_bow(self, kf, kf_mp_ok, kf_fv, f, f_fv):
        return self.m_bow.SearchByBoW(kf, kf_mp_ok, kf_fv, f, f_fv)

    def search_last_frame(self, cf, occupied, lf, lfp, th):
        return self.m_lf.SearchByProjectionLastFrame(cf, occupied, lf, lfp, th, False)

    def search_local_points(self, cf, occupied, mps, th):
        """Tracking::SearchLocalPoints: isInFrustum(0.5) (-> in-view flags, IncreaseVisible)
        and SearchByProjection(F, points, th) with nnratio 0.8."""
        tr = self.m_local.IsInFrustum(cf, mps, 0.5)
        if not np.any(tr["in_view"]):
            return np.full(len(cf.keys), -1, np.int32), 0, tr["in_view"].astype(bool)
        m, n = self.m_local.SearchByProjection(cf, occupied, mps, tr, th)
        return m, n, tr["in_view"].astype(bool)

    def search_for_triangulation(self, kf1, has_mp1, fv1, kf2, has_mp2, fv2, F12):
        """ORBmatcher(0.6, false).SearchForTriangulation(pKF1, pKF2, F12, pairs, false)."""
        return self.m_tri.SearchForTriangulation(kf1, has_mp1, fv1, kf2, has_mp2, fv2, F12, False)

    def fuse_search(self, kf, mps, in_kf, th=3.0):
        """The search of ORBmatcher::Fuse(pKF, vpMapPoints, th) -> (best_idx, best_dist)."""
        bi, bd, _ = self.m_util.FuseSearch(kf, mps, in_kf, th)
        return bi, bd

    def pose_optimization(self, cf, match_lf=None, lf_points=None, match_mp=None, mps=None):
        from .types import POSE_FRAME_DTYPE
        mp, keep = frame_mappoints(match_lf, lf_points, match_mp, mps)
        rec = np.zeros(1, POSE_FRAME_DTYPE)
        out = np.zeros(max(len(cf.keys), 1), np.uint8)
        v = cf.view()
        self.pose.PoseOptimization(v, self.inv_level_sigma2, mp, rec, out)
        del keep
        return rec[0]["tcw"].reshape(4, 4).copy(), out[:len(cf.keys)].copy()

    def distinctive(self, obs_desc, obs_off):
        return self.m_util.ComputeDistinctiveDescriptors(obs_desc, obs_off)[1]

    def local_ba(self, problem, stop=None, stop_at_check=-1):
        return self.ba.run(problem, stop, stop_at_check=stop_at_check)

    def close(self):
        for h in (self.ba, self.pose, self.m_tri, self.m_util, self.m_bow, self.m_local, self.m_lf, self.right, self.left):
            h.close()
        if self.vocab is not None:
            self.vocab.close()


def frame_mappoints(match_lf, lf_points, match_mp, mps):
    """orbmi_frame_mappoints over host arrays -> (struct, arrays to keep alive)."""
    from .types import FrameMapPoints
    mp = FrameMapPoints()
    keep = []
    if match_lf is not None:
        match_lf = np.ascontiguousarray(match_lf, np.int32)
        lf_points = np.ascontiguousarray(lf_points)
        keep += [match_lf, lf_points]
        mp.match_lf, mp.lf_points, mp.n_lf_points = match_lf.ctypes.data, lf_points.ctypes.data, len(lf_points)
    if match_mp is not None:
        match_mp = np.ascontiguousarray(match_mp, np.int32)
        mps = np.ascontiguousarray(mps)
        keep += [match_mp, mps]
        mp.match_mp, mp.mps, mp.n_mps = match_mp.ctypes.data, mps.ctypes.data, len(mps)
    return mp, keep


class StereoSLAM:
    """System(strSettingsFile, STEREO) + Tracking + a synchronous LocalMapping over a backend.

    TrackStereo(imLeft, imRight, timestamp) -> Tcw (4x4 float32, or None while not
    initialised / lost), as System::TrackStereo returns mCurrentFrame.mTcw."""

    def __init__(self, settings, backend=None, device: int = 0, vocabulary=None, local_ba: bool = True,
                 local_mapping: bool = True):
        from .settings import Settings, load_settings
        self.settings = settings if isinstance(settings, Settings) else load_settings(settings)
        s = self.settings
        if s.width <= 0 or s.height <= 0:
            raise ValueError("settings need Camera.width / Camera.height")
        self.cam = s.camera
        self.backend = backend if backend is not None else GpuBackend(s, device, vocabulary)
        if hasattr(self.backend, "bind_camera"):
            self.backend.bind_camera(self.cam)
        self.use_local_ba = local_ba
        # LocalMapping::Run in full (MapPointCulling, CreateNewMapPoints, SearchInNeighbors,
        # KeyFrameCulling); False keeps ProcessNewKeyFrame + MapPointCulling + LocalBA only
        self.local_mapping_full = local_mapping
        sf = np.asarray(self.backend.scale_factors, np.float32)
        self.level_sigma2 = np.ascontiguousarray(sf * sf, np.float32)   # mvLevelSigma2
        self.recent_mps: list[MapPoint] = []   # mlpRecentAddedMapPoints
        self.state = NO_IMAGES_YET
        self.keyframes: list[KeyFrame] = []
        self.mappoints: list[MapPoint] = []
        self.frame_count = 0
        self.last_frame: TrackedFrame | None = None
        self.velocity = None
        self.ref_kf: KeyFrame | None = None
        self.last_kf_frame_id = 0
        self.last_reloc_frame_id = 0
        self.local_kfs: list[KeyFrame] = []
        self.local_mps: list[MapPoint] = []
        self.matches_inliers = 0
        # mlRelativeFramePoses, mlpReferences, mlFrameTimes, mlbLost (src/Tracking.cc:557-580)
        self.rel_poses, self.references, self.frame_times, self.lost = [], [], [], []
        self.stats = []   # per frame: dict of the Tracking counters
        self.ba_log = []  # per LocalBundleAdjustment: graph size and erased observations
        # per keyframe and LocalMapping stage: (keyframe, stage, schedule event, a, b, c) as the
        # native loop's orbmi_slam_get_keyframe_state_log records it (include/orbmi_debug.h)
        self.kf_state = []
        self._state_expect = None  # replay: the recorded rows still to be matched
        self._sched_k = -1         # replay: the schedule event being run
        self._fuse_ops = 0
        # the concurrent LocalMapping of a replayed schedule (replay_schedule): the keyframe queue
        # (mlNewKeyFrames), !AcceptKeyFrames, mbAbortBA and the recorded LocalBA stop checks
        self._concurrent = False
        self._queue = []
        self._busy = False
        self._abort = False
        self._ba_stop_at = None   # kf -> the pbStopFlag check a LocalBA stops at (-1: none)

    # ---- System::TrackStereo ----------------------------------------------------------------
    def TrackStereo(self, imLeft, imRight, timestamp: float):
        keys, desc, u_right, depth = self.backend.extract_stereo(imLeft, imRight)
        n = len(keys)
        cf = TrackedFrame(self.frame_count, float(timestamp), keys, desc.reshape(-1, 32), u_right, depth,
                          map_points=[None] * n, outlier=np.zeros(n, bool))
        self.frame_count += 1
        self._track(cf)
        return None if cf.tcw is None else cf.tcw.copy()

    @staticmethod
    def _drain(gen):
        """Run a stage generator to its end (synchronous use: the yields are the native loop's
        lock releases, nothing runs in between)."""
        try:
            while True:
                next(gen)
        except StopIteration as e:
            return e.value

    def _frame(self, f: TrackedFrame, tcw=None) -> Frame:
        return Frame(f.keys, f.desc, f.u_right, f.tcw if tcw is None else tcw, self.cam, self.backend.scale_factors,
                     self.cam.width, self.cam.height)

    def _track(self, cf: TrackedFrame):
        return self._drain(self._track_gen(cf))

    def _track_gen(self, cf: TrackedFrame):
        """Tracking::Track for a stereo sensor in SLAM mode (src/Tracking.cc:287-581); a generator
        that yields where the native loop releases the map lock (T_*)."""
        if self.state == NO_IMAGES_YET:
            self.state = NOT_INITIALIZED
        st = {"frame": cf.id, "n": cf.n}
        if self.state == NOT_INITIALIZED:
            self._stereo_initialization(cf)
            st["init"] = self.state == OK
            if self.state != OK:
                self.stats.append(st)
                return
            ok = True
        else:
            if self.state == OK:
                self._check_replaced_in_last_frame()
                if self.velocity is None or cf.id < self.last_reloc_frame_id + 2:
                    ok = yield from self._track_reference_kf(cf, st)
                else:
                    ok = yield from self._track_motion_model(cf, st)
                    if not ok:
                        ok = yield from self._track_reference_kf(cf, st)
            else:
                ok = False   # Relocalization is out of scope
            cf.ref_kf = self.ref_kf
            if ok:
                ok = yield from self._track_local_map(cf, st)
            self.state = OK if ok else LOST
            if ok:
                if self.last_frame.tcw is not None:
                    self.velocity = _mul(cf.tcw, pose_inverse(self.last_frame.tcw))
                else:
                    self.velocity = None
                for i, mp in enumerate(cf.map_points):   # clean VO matches (:504-513)
                    if mp is not None and mp.nobs < 1:
                        cf.outlier[i] = False
                        cf.map_points[i] = None
                if self._need_new_keyframe(cf, st):
                    self._create_new_keyframe(cf)
                for i, mp in enumerate(cf.map_points):   # (:535-539)
                    if mp is not None and cf.outlier[i]:
                        cf.map_points[i] = None
            # Reset if the camera gets lost soon after initialisation (src/Tracking.cc:540-551)
            if self.state == LOST and sum(1 for k in self.keyframes if not k.bad) <= 5:
                if self._concurrent:
                    raise NotImplementedError("replay_schedule: a run with a Tracking::Reset")
                self._reset()
                st["reset"] = 1
                st["state"] = self.state
                st["keyframes"] = 0
                st["mappoints"] = 0
                self.stats.append(st)
                return
            if cf.ref_kf is None:
                cf.ref_kf = self.ref_kf
        self.last_frame = cf
        if cf.tcw is not None:
            self.rel_poses.append(_mul(cf.tcw, pose_inverse(cf.ref_kf.tcw)))
            self.references.append(self.ref_kf)
            self.frame_times.append(cf.timestamp)
            self.lost.append(self.state == LOST)
        elif self.rel_poses:
            self.rel_poses.append(self.rel_poses[-1])
            self.references.append(self.references[-1])
            self.frame_times.append(self.frame_times[-1])
            self.lost.append(self.state == LOST)
        st["state"] = self.state
        st["keyframes"] = len(self.keyframes)
        st["mappoints"] = sum(1 for m in self.mappoints if not m.bad)
        self.stats.append(st)

    def _reset(self):
        """Tracking::Reset (src/Tracking.cc:1780-1826): map, tracking state, frame / keyframe ids
        and the trajectory lists start over; the next frame initialises again."""
        self.state = NO_IMAGES_YET
        self.keyframes, self.mappoints, self.recent_mps = [], [], []
        self.frame_count = 0
        self.last_frame = None
        self.velocity = None
        self.ref_kf = None
        self.last_kf_frame_id = 0
        self.last_reloc_frame_id = 0
        self.local_kfs, self.local_mps = [], []
        self.matches_inliers = 0
        self.rel_poses, self.references, self.frame_times, self.lost = [], [], [], []

    # ---- initialisation and keyframes ---------------------------------------------------------
    def _new_keyframe(self, cf: TrackedFrame) -> KeyFrame:
        kf = KeyFrame(len(self.keyframes), cf.id, cf.timestamp, cf.tcw.copy(), cf.keys, cf.desc, cf.u_right,
                      cf.depth, self.backend.inv_level_sigma2, self.backend.scale_factors, self.cam,
                      list(cf.map_points), feat_vec=cf.feat_vec)
        return kf

    def _unproject(self, f: TrackedFrame, idx: np.ndarray) -> np.ndarray:
        """Frame::UnprojectStereo (src/Frame.cc:701-715) in float32."""
        c = self.cam
        z = f.depth[idx].astype(np.float32)
        invfx, invfy = np.float32(1.0) / np.float32(c.fx), np.float32(1.0) / np.float32(c.fy)
        x = ((f.keys["x"][idx] - np.float32(c.cx)) * z * invfx).astype(np.float32)
        y = ((f.keys["y"][idx] - np.float32(c.cy)) * z * invfy).astype(np.float32)
        Twc = pose_inverse(f.tcw)
        pc = np.stack([x, y, z], 0).astype(np.float64)
        # mRwc*x3Dc+mOw is one cv::gemm(Rwc, x3Dc, 1, Ow, 1): Ow added before the one rounding
        return (Twc[:3, :3].astype(np.float64) @ pc + Twc[:3, 3:4].astype(np.float64)).T.astype(np.float32)

    def _create_points(self, kf: KeyFrame, cf: TrackedFrame, idx: list):
        """new MapPoint(x3D, pKF, pMap) + AddObservation + AddMapPoint + ComputeDistinctive +
        UpdateNormalAndDepth for the keypoints `idx` (src/Tracking.cc:602-616, :1308-1320)."""
        if not idx:
            return
        X = self._unproject(cf, np.asarray(idx))
        for j, i in enumerate(idx):
            mp = MapPoint(len(self.mappoints), X[j].copy(), kf, first_kf_id=kf.id)
            mp.add_observation(kf, i)
            kf.map_points[i] = mp
            mp.desc = cf.desc[i].copy()   # ComputeDistinctiveDescriptors of one observation
            self.mappoints.append(mp)
            cf.map_points[i] = mp
        update_normals_and_depths([cf.map_points[i] for i in idx])

    def _stereo_initialization(self, cf: TrackedFrame):
        """Tracking::StereoInitialization (src/Tracking.cc:584-636)."""
        if cf.n <= 500:
            return
        cf.tcw = np.eye(4, dtype=np.float32)
        kf = self._new_keyframe(cf)
        self.keyframes.append(kf)
        self._create_points(kf, cf, [i for i in range(cf.n) if cf.depth[i] > 0])
        self._insert_keyframe(kf)
        self.last_kf_frame_id = cf.id
        self.local_kfs = [kf]
        self.local_mps = [m for m in self.mappoints if not m.bad]
        self.ref_kf = kf
        cf.ref_kf = kf
        self.last_frame = cf
        self.state = OK

    def _need_new_keyframe(self, cf: TrackedFrame, st) -> bool:
        """Tracking::NeedNewKeyFrame (src/Tracking.cc:1140-1249); LocalMapping is idle when it
        runs synchronously, else AcceptKeyFrames / InterruptBA / KeyframesInQueue() < 3."""
        s = self.settings
        nkfs = self._keyframes_in_map()
        if cf.id < self.last_reloc_frame_id + s.max_frames and nkfs > s.max_frames:
            return False
        min_obs = 2 if nkfs <= 2 else 3
        n_ref = self.ref_kf.tracked_map_points(min_obs)
        close = (cf.depth > 0) & (cf.depth < s.th_depth)
        tracked = np.array([mp is not None for mp in cf.map_points], bool) & ~cf.outlier
        n_tracked_close = int(np.sum(close & tracked))
        n_non_tracked_close = int(np.sum(close & ~tracked))
        need_close = n_tracked_close < 100 and n_non_tracked_close > 70
        th_ref = 0.4 if nkfs < 2 else 0.75
        idle = not self._busy
        c1a = cf.id >= self.last_kf_frame_id + s.max_frames
        c1b = cf.id >= self.last_kf_frame_id + s.min_frames and idle
        c1c = self.matches_inliers < n_ref * 0.25 or need_close
        c2 = (self.matches_inliers < n_ref * np.float32(th_ref) or need_close) and self.matches_inliers > 15
        st["need_kf"] = bool((c1a or c1b or c1c) and c2)
        if not st["need_kf"]:
            return False
        if idle:
            return True
        self._abort = True                # mpLocalMapper->InterruptBA()
        return len(self._queue) < 3       # stereo: KeyframesInQueue() < 3

    def _create_new_keyframe(self, cf: TrackedFrame):
        """Tracking::CreateNewKeyFrame for stereo (src/Tracking.cc:1251-1330)."""
        kf = self._new_keyframe(cf)
        self.keyframes.append(kf)
        self.ref_kf = kf
        cf.ref_kf = kf
        order = sorted(((float(cf.depth[i]), i) for i in range(cf.n) if cf.depth[i] > 0))
        new, npts = [], 0
        for z, i in order:
            mp = cf.map_points[i]
            create = mp is None or mp.nobs < 1
            if create and mp is not None:
                cf.map_points[i] = None
                kf.map_points[i] = None
            if create:
                new.append(i)
            npts += 1
            if z > self.settings.th_depth and npts > 100:
                break
        self._create_points(kf, cf, new)
        self._insert_keyframe(kf)
        self.last_kf_frame_id = cf.id

    def _insert_keyframe(self, kf: KeyFrame):
        """LocalMapping::InsertKeyFrame: run it now (synchronous), or queue it for the mapping
        thread and interrupt its BA (src/LocalMapping.cc:130-135)."""
        if not self._concurrent:
            self._drain(self._local_mapping_gen(kf))
            return
        self._queue.append(kf)
        self._abort = True

    # ---- LocalMapping -------------------------------------------------------------------------
    # The stages are generators that yield where the native loop releases its map lock (L_*),
    # with the same state changes between two yields as csrc/slam.cpp, so that a schedule
    # recorded from the native concurrent run replays here (replay_schedule); synchronously they
    # are drained and nothing runs in between.
    def _distinctive(self, mps: list):
        return self._drain(self._distinctive_gen(mps))

    def _obs_rows(self, mps: list):
        """The observation descriptors of the points (CSR, keyframe-id order, bad keyframes out)."""
        rows, off = [], [0]
        for mp in mps:
            for kf in sorted(mp.observations, key=lambda k: k.id):
                if not kf.bad:
                    rows.append(kf.desc[mp.observations[kf]])
            off.append(len(rows))
        return rows, off

    def _distinctive_gen(self, mps: list):
        """MapPoint::ComputeDistinctiveDescriptors for a batch of points (src/MapPoint.cc:247-316)
        on the backend: descriptors of the non-bad observing keyframes, keyframe-id order."""
        rows, off = self._obs_rows(mps)
        if not rows:
            return
        d = self.backend.distinctive(np.asarray(rows, np.uint8), np.asarray(off, np.int32))
        yield L_DISTINCTIVE, -1
        for j, mp in enumerate(mps):
            if off[j + 1] > off[j]:
                mp.desc = np.asarray(d[j], np.uint8).copy()

    def _keyframes_in_map(self) -> int:
        return sum(1 for k in self.keyframes if not k.bad)   # Map::KeyFramesInMap

    def _queued(self) -> bool:
        """LocalMapping::CheckNewKeyFrames (always false when synchronous)."""
        return self._concurrent and len(self._queue) > 0

    def _local_mapping(self, kf: KeyFrame):
        return self._drain(self._local_mapping_gen(kf))

    def _local_mapping_gen(self, kf: KeyFrame):
        """LocalMapping::Run for one keyframe (src/LocalMapping.cc:47-128): ProcessNewKeyFrame,
        MapPointCulling, CreateNewMapPoints, SearchInNeighbors unless a keyframe is queued,
        LocalBundleAdjustment (more than 2 keyframes) and KeyFrameCulling unless one is queued."""
        # ProcessNewKeyFrame (:152-211); as the native loop: the observations first, then
        # ComputeBoW and the updated points' ComputeDistinctiveDescriptors in one window with the
        # map lock released (the transform reads only the keyframe's descriptors)
        need_bow = self.backend_has_bow() and kf.feat_vec is None
        updated = []
        for i, mp in enumerate(kf.map_points):
            if mp is None or mp.bad:
                continue
            if kf not in mp.observations:
                mp.add_observation(kf, i)
                updated.append(mp)
            else:   # the new stereo points the Tracking inserted
                self.recent_mps.append(mp)
        update_normals_and_depths(updated)
        rows, off = self._obs_rows(updated)
        if need_bow or rows:
            fv = self.backend.compute_bow(kf.desc) if need_bow else None
            d = self.backend.distinctive(np.asarray(rows, np.uint8), np.asarray(off, np.int32)) if rows else None
            yield (L_BOW, kf.id) if need_bow else (L_DISTINCTIVE, -1)
            if need_bow and kf.feat_vec is None:  # (Tracking may have computed it meanwhile: the same)
                kf.feat_vec = fv
            if rows:
                for j, mp in enumerate(updated):
                    if off[j + 1] > off[j]:
                        mp.desc = np.asarray(d[j], np.uint8).copy()
        kf.update_connections()
        fv = kf.feat_vec
        if fv is None:
            self._log_state(kf, KF_STATE_PROCESS, -1, FNV0, _slot_hash(kf))
        else:
            h = _fnv(_fnv(_fnv(FNV0, fv.node_id), fv.off), fv.feat)
            self._log_state(kf, KF_STATE_PROCESS, getattr(fv, "n_words", -1), h, _slot_hash(kf))
        self._map_point_culling(kf)
        owed2 = []   # SearchInNeighbors' last ComputeDistinctiveDescriptors, done in LocalBA's window
        if self.local_mapping_full:
            n0 = len(self.mappoints)
            owed = (yield from self._create_new_map_points_gen(kf)) or []
            self._log_state(kf, KF_STATE_CREATE, len(self.mappoints) - n0, len(self.mappoints), _slot_hash(kf))
            if self._queued():
                yield from self._distinctive_gen(owed)
            else:
                self._fuse_ops = 0
                owed2 = yield from self._search_in_neighbors_gen(kf, owed)
                filled = sum(1 for mp in kf.map_points if mp is not None)
                self._log_state(kf, KF_STATE_FUSE, self._fuse_ops, filled, _slot_hash(kf))
        self._abort = False
        if not self._queued():
            if self.use_local_ba and self._keyframes_in_map() > 2:
                yield from self._local_bundle_adjustment_gen(kf, owed2)
            else:
                yield from self._distinctive_gen(owed2)
            if self.local_mapping_full:
                self._keyframe_culling(kf)
        else:
            yield from self._distinctive_gen(owed2)

    def _log_state(self, kf: KeyFrame, stage: int, a: int, b: int, c: int):
        """The per-keyframe state record (orbmi_slam_kf_state); in a replay, checked against the
        native run's record at the same point, so a divergence is named by its first keyframe and
        stage instead of by a lock label many events later."""
        row = (kf.id, stage, self._sched_k, int(a), _i32(b), _i32(c))
        self.kf_state.append(row)
        if self._state_expect is None:
            return
        want = next(self._state_expect, None)
        if want is None or tuple(want) != row:
            names = ("ProcessNewKeyFrame", "CreateNewMapPoints", "SearchInNeighbors")
            raise ScheduleMismatch(f"keyframe {kf.id}, after {names[stage]}: the native run recorded {want} "
                                   f"(keyframe, stage, event, a, b, c), this logic {row}")

    def _map_point_culling(self, kf: KeyFrame):
        """LocalMapping::MapPointCulling (src/LocalMapping.cc:219-263), stereo: nThObs = 3."""
        keep = []
        for mp in self.recent_mps:
            if mp.bad:
                continue
            if mp.found_ratio() < np.float32(0.25):
                mp.set_bad()
            elif kf.id - mp.first_kf_id >= 2 and mp.nobs <= 3:
                mp.set_bad()
            elif kf.id - mp.first_kf_id >= 3:
                continue
            else:
                keep.append(mp)
        self.recent_mps = keep

    def _tri_view(self, kf: KeyFrame):
        """orbmi_tri_keyframe of a keyframe (host arrays kept alive by the returned tuple)."""
        from .types import TriKeyFrame
        tcw = np.ascontiguousarray(kf.tcw, np.float32)
        keys = np.ascontiguousarray(kf.keys_un)
        ur = np.ascontiguousarray(kf.u_right, np.float32)
        depth = np.ascontiguousarray(kf.depth, np.float32)
        sig2 = self.level_sigma2
        c = self.cam
        v = TriKeyFrame(tcw.ctypes.data, keys.ctypes.data, ur.ctypes.data, depth.ctypes.data, c.fx, c.fy, c.cx, c.cy,
                        c.bf, np.float32(np.float32(c.bf) / np.float32(c.fx)), sig2.ctypes.data,
                        self.backend.scale_factors.ctypes.data)
        return v, (tcw, keys, ur, depth, sig2)

    def _kf_frame(self, kf: KeyFrame) -> Frame:
        return Frame(kf.keys_un, kf.desc, kf.u_right, kf.tcw, self.cam, self.backend.scale_factors,
                     self.cam.width, self.cam.height)

    def _create_new_map_points_gen(self, kf: KeyFrame):
        """LocalMapping::CreateNewMapPoints (src/LocalMapping.cc:290-577), stereo: the 10 best
        covisible keyframes, baseline >= mb, SearchForTriangulation (0.6, no orientation check)
        on the backend, the triangulation / acceptance geometry on the host
        (orbmi_triangulate_matches), new points with both observations.  As the native loop does
        it in one device call: every pair's search and triangulation first (a keypoint an earlier
        pair triangulated is not searched again: the reference's `if (pMP1) continue`), then the
        new points pair by pair with CheckNewKeyFrames between pairs (:331).  Their
        ComputeDistinctiveDescriptors (per point: the same as pair by pair) is returned as owed, to
        the caller, which does it with SearchInNeighbors' first device call."""
        import ctypes as C
        from ._capi import check, lib
        if kf.feat_vec is None:
            return   # (no vocabulary: no FeatureVector, no searches)
        ow1 = kf.Ow
        v1, keep1 = self._tri_view(kf)
        mb = np.float32(np.float32(self.cam.bf) / np.float32(self.cam.fx))
        pairs = []
        for i, kf2 in enumerate(kf.best_covisibility(10)):
            d = (kf2.Ow - ow1).astype(np.float32).astype(np.float64)
            baseline = np.float32(np.sqrt(np.sum(d * d)))
            if baseline < mb or kf2.feat_vec is None:
                continue
            v2, keep2 = self._tri_view(kf2)
            F12 = np.zeros(9, np.float32)
            check("orbmi_compute_f12", lib().orbmi_compute_f12(C.addressof(v1), C.addressof(v2), F12.ctypes.data))
            has2 = np.array([mp is not None for mp in kf2.map_points], np.uint8)
            pairs.append((i, kf2, v2, keep2, F12, has2))
        if not pairs:
            return
        has1 = np.array([mp is not None for mp in kf.map_points], np.uint8)
        results = []
        for i, kf2, v2, keep2, F12, has2 in pairs:
            m12, _ = self.backend.search_for_triangulation(self._kf_frame(kf), has1, kf.feat_vec, self._kf_frame(kf2),
                                                           has2, kf2.feat_vec, F12.reshape(3, 3))
            idx1 = np.nonzero(np.asarray(m12) >= 0)[0].astype(np.int32)
            idx2 = np.asarray(m12, np.int32)[idx1]
            x3d = np.zeros((len(idx1), 3), np.float32)
            ok = np.zeros(len(idx1), np.uint8)
            if len(idx1):
                check("orbmi_triangulate_matches", lib().orbmi_triangulate_matches(
                    C.addressof(v1), C.addressof(v2), idx1.ctypes.data, idx2.ctypes.data, len(idx1), x3d.ctypes.data,
                    ok.ctypes.data))
                has1[idx1[ok != 0]] = 1
            results.append((i, kf2, idx1, idx2, ok, x3d))
        yield L_CREATE, kf.id
        fresh = []
        for i, kf2, idx1, idx2, ok, x3d in results:
            if i > 0 and self._queued():   # src/LocalMapping.cc:331
                break
            for k in np.nonzero(ok)[0]:
                i1, i2 = int(idx1[k]), int(idx2[k])
                mp = MapPoint(len(self.mappoints), x3d[k].copy(), kf, first_kf_id=kf.id,
                              desc=np.zeros(32, np.uint8), normal=np.zeros(3, np.float32))
                mp.add_observation(kf, i1)
                mp.add_observation(kf2, i2)
                kf.map_points[i1] = mp
                kf2.map_points[i2] = mp
                self.mappoints.append(mp)
                self.recent_mps.append(mp)
                fresh.append(mp)
        update_normals_and_depths(fresh)
        del keep1
        return fresh

    def _mp_fuse_records(self, mps: list) -> np.ndarray:
        rec = np.zeros(len(mps), MAPPOINT_DTYPE)
        if not mps:
            return rec
        rec["pos"] = np.array([mp.pos for mp in mps], np.float32)
        rec["normal"] = np.array([mp.normal for mp in mps], np.float32)
        rec["max_distance"] = np.array([mp.max_distance for mp in mps], np.float32)
        rec["min_distance"] = np.array([mp.min_distance for mp in mps], np.float32)
        rec["desc"] = np.array([mp.desc for mp in mps], np.uint8)
        rec["flags"] = np.array([(MP_BAD if mp.bad else 0) | (MP_HAS_OBS if mp.nobs > 0 else 0) for mp in mps],
                                np.uint32)
        return rec

    def _fuse_search_gen(self, kf: KeyFrame, pts: list):
        """The search of ORBmatcher::Fuse(pKF, points, 3.0) on the backend -> best keypoint per point."""
        in_kf = np.array([kf in mp.observations for mp in pts], np.uint8)
        best, _ = self.backend.fuse_search(self._kf_frame(kf), self._mp_fuse_records(pts), in_kf, 3.0)
        yield L_FUSE, kf.id
        return np.asarray(best, np.int32).copy()

    def _fuse_replay(self, kf: KeyFrame, pts: list, best, dirty: set):
        """The map updates of ORBmatcher::Fuse (src/ORBmatcher.cc:1096-1124) in list order
        (counted in _fuse_ops for the state record)."""
        for mp, b in zip(pts, best):
            if mp.bad or kf in mp.observations or b < 0:
                continue
            b = int(b)
            mp_in_kf = kf.map_points[b]
            if mp_in_kf is not None:
                if not mp_in_kf.bad:
                    if mp_in_kf.nobs > mp.nobs:
                        if mp.replace(mp_in_kf):
                            dirty.add(mp_in_kf)
                            self._fuse_ops += 1
                    elif mp_in_kf.replace(mp):
                        dirty.add(mp)
                        self._fuse_ops += 1
            else:
                mp.add_observation(kf, b)
                kf.map_points[b] = mp
                self._fuse_ops += 1

    def _fuse_gen(self, kf: KeyFrame, mps: list, dirty: set):
        """ORBmatcher::Fuse(pKF, vpMapPoints, 3.0) (src/ORBmatcher.cc:977-1127): the search for
        every point on the backend, then the map updates in list order; first the descriptors
        MapPoint::Replace still owes (src/MapPoint.cc:212)."""
        due = sorted((m for m in dirty if not m.bad), key=lambda m: m.id)
        dirty.clear()
        pts = [mp for mp in mps if mp is not None]
        if not pts:
            yield from self._distinctive_gen(due)
            return
        rows, off = self._obs_rows(due)
        if not rows:
            best = yield from self._fuse_search_gen(kf, pts)
            self._fuse_replay(kf, pts, best, dirty)
            return
        # the native loop's one device call (orbmi_fuse_search_refresh): the owed descriptors,
        # then the search with each due point's new descriptor
        newd = self.backend.distinctive(np.asarray(rows, np.uint8), np.asarray(off, np.int32))
        at = {m.id: d for d, m in enumerate(due) if off[d + 1] > off[d]}
        rec = self._mp_fuse_records(pts)
        for j, mp in enumerate(pts):
            if mp.id in at:
                rec["desc"][j] = np.asarray(newd[at[mp.id]], np.uint8)
        in_kf = np.array([kf in mp.observations for mp in pts], np.uint8)
        best, _ = self.backend.fuse_search(self._kf_frame(kf), rec, in_kf, 3.0)
        best = np.asarray(best, np.int32).copy()
        yield L_FUSE, kf.id
        for d, m in enumerate(due):
            if off[d + 1] > off[d]:
                m.desc = np.asarray(newd[d], np.uint8).copy()
        self._fuse_replay(kf, pts, best, dirty)

    def _fuse_targets_gen(self, targets: list, lst: list, dirty: set, owed=()):
        """Fuse(target, the keyframe's points) for every target in order (src/LocalMapping.cc:
        620-628), as csrc/slam.cpp fuse_targets runs it: every target searched on the records as
        they are before the first one, then per target: the owed descriptors of listed points
        (and those points searched again against this and the later targets), the points whose
        record an earlier replay changed searched again, the replay.  Results are the
        target-by-target loop's; the state between the steps is the native loop's."""
        pts = [mp for mp in lst if mp is not None]
        nt, npts = len(targets), len(pts)
        if nt == 0 or npts == 0:
            yield from self._distinctive_gen(list(owed))
            return
        rec0 = self._mp_fuse_records(pts)
        # the descriptors CreateNewMapPoints owes, in the batch's device call (the searches read them)
        due = [m for m in owed if not m.bad]
        orows, ooff = self._obs_rows(due)
        if orows:
            odesc = self.backend.distinctive(np.asarray(orows, np.uint8), np.asarray(ooff, np.int32))
            at = {m.id: d for d, m in enumerate(due) if ooff[d + 1] > ooff[d]}
            for j, mp in enumerate(pts):
                if mp.id in at:
                    rec0["desc"][j] = np.asarray(odesc[at[mp.id]], np.uint8)
        best = []
        for t in targets:
            in0 = np.array([t in mp.observations for mp in pts], np.uint8)
            bi, _ = self.backend.fuse_search(self._kf_frame(t), rec0, in0, 3.0)
            best.append(np.asarray(bi, np.int32).copy())
        yield L_FUSE_BATCH, -1
        if orows:
            for d, m in enumerate(due):
                if ooff[d + 1] > ooff[d]:
                    m.desc = np.asarray(odesc[d], np.uint8).copy()
        listed = {}
        for j in range(npts - 1, -1, -1):
            listed[pts[j]] = j
        for t in range(nt):
            kt = targets[t]
            due = []
            for m in sorted(dirty, key=lambda m: m.id):
                if m in listed:
                    if not m.bad:
                        due.append(m)
                    dirty.discard(m)
            if due:
                rows, off = self._obs_rows(due)
                rj, frm = [], []
                for d, m in enumerate(due):
                    for j in range(npts):
                        if pts[j] is m:
                            rj.append(j)
                            frm.append(d if off[d + 1] > off[d] else -1)
                newd = None
                if rows:
                    newd = self.backend.distinctive(np.asarray(rows, np.uint8), np.asarray(off, np.int32))
                rrec = self._mp_fuse_records([pts[j] for j in rj])
                for q, f in enumerate(frm):
                    if f >= 0:
                        rrec["desc"][q] = np.asarray(newd[f], np.uint8)
                for u in range(t, nt):
                    rin = np.array([targets[u] in pts[j].observations for j in rj], np.uint8)
                    bi, _ = self.backend.fuse_search(self._kf_frame(targets[u]), rrec, rin, 3.0)
                    for q, j in enumerate(rj):
                        best[u][j] = int(bi[q])
                yield L_FUSE_REFRESH, t
                for d, m in enumerate(due):
                    if off[d + 1] > off[d]:
                        m.desc = np.asarray(newd[d], np.uint8).copy()
                for j in rj:
                    rec0[j] = self._mp_fuse_records([pts[j]])[0]
            row = best[t]
            redo = [j for j, m in enumerate(pts) if not (m.bad or kt in m.observations)
                    and self._mp_fuse_records([m])[0].tobytes() != rec0[j].tobytes()]
            if redo:
                b2 = yield from self._fuse_search_gen(kt, [pts[j] for j in redo])
                for q, j in enumerate(redo):
                    row[j] = b2[q]
            self._fuse_replay(kt, pts, row, dirty)

    def _search_in_neighbors_gen(self, kf: KeyFrame, owed=()):
        """LocalMapping::SearchInNeighbors (src/LocalMapping.cc:589-674), stereo: nn = 10."""
        targets = []
        for k in kf.best_covisibility(10):
            if k.bad or k.fuse_target_for_kf == kf.id:
                continue
            targets.append(k)
            k.fuse_target_for_kf = kf.id
            for k2 in k.best_covisibility(5):
                if k2.bad or k2.fuse_target_for_kf == kf.id or k2.id == kf.id:
                    continue
                targets.append(k2)
        dirty = set()
        yield from self._fuse_targets_gen(targets, list(kf.map_points), dirty, owed)
        cands = []
        for k in targets:
            for mp in k.map_points:
                if mp is None or mp.bad or mp.fuse_candidate_for_kf == kf.id:
                    continue
                mp.fuse_candidate_for_kf = kf.id
                cands.append(mp)
        yield from self._fuse_gen(kf, cands, dirty)
        dirty.clear()
        pts = [mp for mp in kf.map_points if mp is not None and not mp.bad]
        seen, upd = set(), []
        for mp in pts:   # one update per point (a point may sit at two keypoints after a Replace)
            if id(mp) not in seen:
                seen.add(id(mp))
                upd.append(mp)
        # their ComputeDistinctiveDescriptors is returned to the caller (LocalBA's device window, as
        # the native loop); UpdateNormalAndDepth and UpdateConnections do not read descriptors
        update_normals_and_depths(upd)
        kf.update_connections()
        return upd

    def _keyframe_culling(self, kf: KeyFrame):
        """LocalMapping::KeyFrameCulling (src/LocalMapping.cc:775-841), stereo: close points only;
        a keyframe is redundant when 90 % of them are seen by >= 3 other keyframes at the same or
        a finer scale."""
        th_depth = self.settings.th_depth
        for k in list(kf.covisible):
            if k.id == 0:
                continue
            n_mps = n_red = 0
            for i, mp in enumerate(k.map_points):
                if mp is None or mp.bad:
                    continue
                if k.depth[i] > th_depth or k.depth[i] < 0:
                    continue
                n_mps += 1
                if mp.nobs > 3:
                    level = int(k.keys_un[i]["octave"])
                    n = 0
                    for ki in sorted(mp.observations, key=lambda x: x.id):
                        if ki is k:
                            continue
                        if int(ki.keys_un[mp.observations[ki]]["octave"]) <= level + 1:
                            n += 1
                            if n >= 3:
                                break
                    if n >= 3:
                        n_red += 1
            if n_red > 0.9 * n_mps:
                k.set_bad()

    def backend_has_bow(self) -> bool:
        return getattr(self.backend, "vocab", None) is not None

    def _local_bundle_adjustment_gen(self, kf: KeyFrame, owed=()):
        """Optimizer::LocalBundleAdjustment (src/Optimizer.cc:483-808): graph assembly on the host
        (optimizer.gather_local_ba), optimisation on the backend, write-back under the map lock.
        In a replayed schedule pbStopFlag (mbAbortBA) is the recorded run's: the backend stops at
        the check where that run first saw it raised (orbmi_ba_set_stop_at_check)."""
        from .optimizer import gather_local_ba
        problem, kfs, mps = gather_local_ba(kf)
        owed = list(owed)
        if len(problem.edges) == 0:
            yield from self._distinctive_gen(owed)
            return
        # `owed`: ComputeDistinctiveDescriptors in the same device window (native: one lock release)
        rows, off = self._obs_rows(owed)
        d = self.backend.distinctive(np.asarray(rows, np.uint8), np.asarray(off, np.int32)) if rows else None
        stop_at = -1 if self._ba_stop_at is None else self._ba_stop_at(kf)
        res = self.backend.local_ba(problem, stop_at_check=stop_at)
        yield L_BA, kf.id
        if rows:
            for j, mp in enumerate(owed):
                if off[j + 1] > off[j]:
                    mp.desc = np.asarray(d[j], np.uint8).copy()
        erase = np.asarray(res["erase"], bool)
        self.ba_log.append({"keyframe": kf.id, "keyframes": len(kfs), "points": len(mps),
                            "edges": len(problem.edges), "erased": int(erase.sum()),
                            "iterations": tuple(res["iterations"]), "stop_check": res.get("stop_check", -1),
                            "aborted": res["aborted"]})
        if res["aborted"]:
            return   # src/Optimizer.cc:685-687: stopped before optimising, nothing written back
        for e in np.nonzero(erase)[0]:
            ed = problem.edges[e]
            mp, k = mps[int(ed["point"])], kfs[int(ed["kf"])]
            if k in mp.observations and k.map_points[mp.observations[k]] is mp:
                k.map_points[mp.observations[k]] = None    # KeyFrame::EraseMapPointMatch
            mp.erase_observation(k)
        n_local = 1 + sum(1 for k in kf.covisible if not k.bad)
        for i in range(n_local):
            kfs[i].tcw = np.asarray(res["tcw"][i], np.float32).reshape(4, 4).copy()
        for j, mp in enumerate(mps):
            mp.pos = np.asarray(res["pos"][j], np.float32).copy()
        update_normals_and_depths(mps)

    # ---- replay of a concurrent schedule ------------------------------------------------------
    def _tracking_thread(self, frames):
        """Tracking's side of a concurrent run: per frame the Frame constructor (no shared state),
        then Track() under the map lock (T_FRAME) with its releases."""
        for L, R, ts in frames:
            keys, desc, u_right, depth = self.backend.extract_stereo(L, R)
            n = len(keys)
            cf = TrackedFrame(self.frame_count, float(ts), keys, desc.reshape(-1, 32), u_right, depth,
                              map_points=[None] * n, outlier=np.zeros(n, bool))
            yield T_FRAME, cf.id
            self.frame_count += 1
            yield from self._track_gen(cf)

    def _mapping_thread(self):
        """LocalMapping's thread: each time it takes the map lock it takes the next queued
        keyframe (if any: a reset may have dropped it) and runs LocalMapping::Run for it."""
        while True:
            ev = yield L_JOB, None
            kf = None
            if self._queue:
                kf = self._queue.pop(0)
                self._busy = True   # SetAcceptKeyFrames(false)
            got = -1 if kf is None else kf.id
            if ev is not None and int(ev[2]) != got:
                raise ScheduleMismatch(f"the mapping thread took keyframe {got}, the record {int(ev[2])}")
            if kf is not None:
                yield from self._local_mapping_gen(kf)
            self._busy = False      # SetAcceptKeyFrames(true)

    def replay_schedule(self, frames, schedule, ba_log, kf_state=None):
        """Replay a run of the native loop with the concurrent LocalMapping
        (orbmi_slam_settings.async_local_mapping) on this host logic: `frames` = [(L, R, ts)] as
        handed to TrackStereo, `schedule` = NativeStereoSLAM.schedule() (thread, label, arg per
        acquisition of the map lock, in order), `ba_log` = NativeStereoSLAM.local_ba_log().  The
        two threads' stretches between lock releases run in the recorded order and every
        LocalBA stops at its recorded pbStopFlag check, so the run's decisions and trajectory
        follow from the schedule.  Raises ScheduleMismatch where the record and this logic
        disagree; with `kf_state` (NativeStereoSLAM.keyframe_state_log()) every keyframe's state
        after ProcessNewKeyFrame, CreateNewMapPoints and SearchInNeighbors is compared as it is
        reached, so a mismatch names the first keyframe and stage where the maps part."""
        self._concurrent = True
        if kf_state is not None:
            self._state_expect = iter([tuple(int(x) for x in r) for r in np.asarray(kf_state).reshape(-1, 6)])
        stops = iter([tuple(int(x) for x in r[:2]) for r in np.asarray(ba_log).reshape(-1, 8)])

        def stop_at(kf):
            rec = next(stops, None)
            if rec is None or rec[0] != kf.id:
                raise ScheduleMismatch(f"LocalBA of keyframe {kf.id}, the record has {rec}")
            return rec[1]
        self._ba_stop_at = stop_at
        gens = {0: self._tracking_thread(frames), 1: self._mapping_thread()}
        want = {t: next(g) for t, g in gens.items()}
        for k, (thread, label, arg) in enumerate(np.asarray(schedule).reshape(-1, 3).tolist()):
            w = want.get(thread)
            if w is None or w[0] != label or (w[1] is not None and w[1] != arg):
                raise ScheduleMismatch(f"event {k}: thread {thread} resumes at ({label}, {arg}), "
                                       f"this logic at {w}")
            self._sched_k = k
            try:
                want[thread] = gens[thread].send((thread, label, arg))
            except StopIteration:
                want[thread] = None
        if want[0] is not None:
            raise ScheduleMismatch(f"the record ends with Tracking at {want[0]}")
        if next(stops, None) is not None:
            raise ScheduleMismatch("the record has more LocalBA calls")
        if self._state_expect is not None and next(self._state_expect, None) is not None:
            raise ScheduleMismatch("the record has more keyframe states")
        self._concurrent = False
        self._ba_stop_at = None
        self._state_expect = None
        self._sched_k = -1

    def ba_records(self) -> np.ndarray:
        """ba_log in the layout of NativeStereoSLAM.local_ba_log (keyframe, stop_check, aborted,
        checks, iterations0, iterations1, edges, erased; checks not kept: -1)."""
        return np.array([[b["keyframe"], b["stop_check"], b["aborted"], -1, b["iterations"][0], b["iterations"][1],
                          b["edges"], b["erased"]] for b in self.ba_log], np.int32).reshape(-1, 8)

    # ---- tracking stages --------------------------------------------------------------------
    def _mp_records(self, mps: list, seen: set) -> np.ndarray:
        """orbmi_mappoint records of local map points (include/orbmi.h)."""
        rec = np.zeros(len(mps), MAPPOINT_DTYPE)
        if not mps:
            return rec
        rec["pos"] = np.array([mp.pos for mp in mps], np.float32)
        rec["normal"] = np.array([mp.normal for mp in mps], np.float32)
        rec["max_distance"] = np.array([mp.max_distance for mp in mps], np.float32)
        rec["min_distance"] = np.array([mp.min_distance for mp in mps], np.float32)
        rec["desc"] = np.array([mp.desc for mp in mps], np.uint8)
        rec["flags"] = np.array([(MP_BAD if mp.bad else 0) | (MP_SEEN if id(mp) in seen else 0) |
                                 (MP_HAS_OBS if mp.nobs > 0 else 0) for mp in mps], np.uint32)
        return rec

    def _lf_records(self, lf_mps: list, outlier) -> np.ndarray:
        """orbmi_lastframe_point records of a frame's mvpMapPoints (include/orbmi.h)."""
        rec = np.zeros(len(lf_mps), LFPOINT_DTYPE)
        idx = [i for i, mp in enumerate(lf_mps) if mp is not None]
        if not idx:
            return rec
        pts = [lf_mps[i] for i in idx]
        rec["pos"][idx] = np.array([mp.pos for mp in pts], np.float32)
        rec["desc"][idx] = np.array([mp.desc for mp in pts], np.uint8)
        fl = np.array([LF_HAS_MP | (MP_HAS_OBS if mp.nobs > 0 else 0) for mp in pts], np.uint32)
        if outlier is not None:
            fl |= np.where(np.asarray(outlier)[idx], LF_OUTLIER, 0).astype(np.uint32)
        rec["flags"][idx] = fl
        return rec

    def _discard_outliers(self, cf: TrackedFrame, outlier, seen: set) -> int:
        """The pass after PoseOptimization in TrackReferenceKeyFrame / TrackWithMotionModel
        (src/Tracking.cc:904-917, :1036-1058) -> nmatchesMap."""
        nmap = 0
        for i, mp in enumerate(cf.map_points):
            if mp is None:
                continue
            if outlier[i]:
                cf.map_points[i] = None
                cf.outlier[i] = False
                seen.add(id(mp))   # pMP->mnLastFrameSeen = mCurrentFrame.mnId
            elif mp.nobs > 0:
                nmap += 1
        return nmap

    def _check_replaced_in_last_frame(self):
        """Tracking::CheckReplacedInLastFrame: map points the LocalMapping replaced (Fuse)."""
        lf = self.last_frame
        for i, mp in enumerate(lf.map_points):
            if mp is not None and mp.replaced is not None:
                lf.map_points[i] = mp.replaced

    def _update_last_frame(self):
        """Tracking::UpdateLastFrame (src/Tracking.cc:919-995) in SLAM mode: only the pose."""
        lf = self.last_frame
        lf.tcw = _mul(self.rel_poses[-1], lf.ref_kf.tcw)

    def _track_reference_kf(self, cf: TrackedFrame, st):
        """Tracking::TrackReferenceKeyFrame (src/Tracking.cc:871-917); generator -> ok."""
        cf.feat_vec = self.backend.compute_bow(cf.desc)
        kf = self.ref_kf
        if kf.feat_vec is None:
            kf.feat_vec = self.backend.compute_bow(kf.desc)
        ok_mp = np.array([mp is not None and not mp.bad for mp in kf.map_points], np.uint8)
        kf_mps = list(kf.map_points)   # the keyframe's matches when the search ran
        kfv = Frame(kf.keys_un, kf.desc, kf.u_right, kf.tcw, self.cam, self.backend.scale_factors,
                    self.cam.width, self.cam.height)
        m, n = self.backend.search_by_bow(kfv, ok_mp, kf.feat_vec, self._frame(cf, np.eye(4)), cf.feat_vec)
        yield T_BOW, cf.id
        st["bow_matches"] = n
        st["track"] = "reference_kf"
        if n < 15:
            return False
        cf.map_points = [kf_mps[j] if j >= 0 else None for j in m]
        cf.tcw = self.last_frame.tcw.copy()
        lfp = self._lf_records(kf_mps, None)
        tcw, out = self.backend.pose_optimization(self._frame(cf), np.asarray(m, np.int32), lfp)
        yield T_POSE, cf.id
        cf.tcw = tcw
        cf.outlier = out.astype(bool)
        self._seen = set()
        nmap = self._discard_outliers(cf, cf.outlier.copy(), self._seen)
        st["nmatches_map"] = nmap
        return nmap >= 10

    def _track_motion_model(self, cf: TrackedFrame, st):
        """Tracking::TrackWithMotionModel (src/Tracking.cc:997-1063); generator -> ok.  The
        searches (the retry at 2 th when fewer than 20 matched) and PoseOptimization run on the
        inputs as they are when the stage starts (the native loop's one device-resident window)."""
        self._update_last_frame()
        lf = self.last_frame
        cf.tcw = _mul(self.velocity, lf.tcw)
        lfp = self._lf_records(lf.map_points, lf.outlier)
        occ = np.zeros(cf.n, np.uint8)
        lfv = self._frame(lf)
        th = 7.0   # stereo (src/Tracking.cc:1011-1014)
        m, n = self.backend.search_last_frame(self._frame(cf), occ, lfv, lfp, th)
        if n < 20:
            m, n = self.backend.search_last_frame(self._frame(cf), occ, lfv, lfp, 2 * th)
        if n >= 20:
            tcw, out = self.backend.pose_optimization(self._frame(cf), np.asarray(m, np.int32), lfp)
        yield T_LF, cf.id
        st["track"] = "motion_model"
        st["lf_matches"] = n
        if n < 20:
            return False
        cf.map_points = [lf.map_points[j] if j >= 0 else None for j in m]
        cf.tcw = tcw
        cf.outlier = out.astype(bool)
        self._seen = set()
        nmap = self._discard_outliers(cf, cf.outlier.copy(), self._seen)
        st["nmatches_map"] = nmap
        return nmap >= 10

    def _update_local_keyframes(self, cf: TrackedFrame):
        """Tracking::UpdateLocalKeyFrames (src/Tracking.cc:1452-1580), including its early exit
        of the outer loop after a parent is added."""
        counter: dict = {}
        for i, mp in enumerate(cf.map_points):
            if mp is None:
                continue
            if mp.bad:
                cf.map_points[i] = None
                continue
            for kf in mp.observations:
                counter[kf] = counter.get(kf, 0) + 1
        if not counter:
            return
        best, kfmax = 0, None
        local, mark = [], set()
        for kf in sorted(counter, key=lambda k: k.id):
            if kf.bad:
                continue
            if counter[kf] > best:
                best, kfmax = counter[kf], kf
            local.append(kf)
            mark.add(id(kf))
        i = 0
        while i < len(local):
            if len(local) > 80:
                break
            kf = local[i]
            i += 1
            for nb in kf.best_covisibility(10):
                if not nb.bad and id(nb) not in mark:
                    local.append(nb)
                    mark.add(id(nb))
                    break
            for ch in sorted(kf.children, key=lambda k: k.id):
                if not ch.bad and id(ch) not in mark:
                    local.append(ch)
                    mark.add(id(ch))
                    break
            p = kf.parent
            if p is not None and id(p) not in mark:
                local.append(p)
                mark.add(id(p))
                break
        self.local_kfs = local
        if kfmax is not None:
            self.ref_kf = kfmax
            cf.ref_kf = kfmax

    def _update_local_points(self):
        """Tracking::UpdateLocalPoints (src/Tracking.cc:1421-1450)."""
        out, mark = [], set()
        for kf in self.local_kfs:
            for mp in kf.map_points:
                if mp is None or id(mp) in mark or mp.bad:
                    continue
                out.append(mp)
                mark.add(id(mp))
        self.local_mps = out

    def _track_local_map(self, cf: TrackedFrame, st):
        """Tracking::TrackLocalMap (src/Tracking.cc:1075-1104) with UpdateLocalMap and
        SearchLocalPoints (:1345-1420); generator -> ok.  SearchLocalPoints and PoseOptimization run
        on the records as they are when the stage starts (the native loop's one window)."""
        self._update_local_keyframes(cf)
        self._update_local_points()
        seen = getattr(self, "_seen", set())
        occ = np.zeros(cf.n, np.uint8)
        for i, mp in enumerate(cf.map_points):   # SearchLocalPoints' first loop
            if mp is None:
                continue
            if mp.bad:
                cf.map_points[i] = None
            else:
                mp.visible += 1   # IncreaseVisible
                seen.add(id(mp))
                occ[i] = 1 if mp.nobs > 0 else 0
        mps = self.local_mps
        rec = self._mp_records(mps, seen)
        m_mp, nl, in_view = self.backend.search_local_points(self._frame(cf), occ, rec, 1.0)
        m_lf = np.full(cf.n, -1, np.int32)
        cur = list(cf.map_points)
        for i, j in enumerate(m_mp):
            if j >= 0:
                cur[i] = mps[j]
        # PoseOptimization over the frame's map points: one record per keypoint
        lfp = self._lf_records(cur, None)
        for i, mp in enumerate(cur):
            if mp is not None:
                m_lf[i] = i
        tcw, out = self.backend.pose_optimization(self._frame(cf), m_lf, lfp)
        yield T_LOCAL, cf.id
        for j in np.nonzero(np.asarray(in_view))[0]:   # isInFrustum -> IncreaseVisible
            mps[int(j)].visible += 1
        st["local_map_points"] = len(mps)
        st["local_matches"] = nl
        cf.tcw = tcw
        cf.map_points = cur
        cf.outlier = out.astype(bool)
        inliers = 0
        for i, mp in enumerate(cf.map_points):   # (:1087-1101)
            if mp is None:
                continue
            if not cf.outlier[i]:
                mp.found += 1   # IncreaseFound
                if mp.nobs > 0:
                    inliers += 1
            elif cf.u_right[i] >= 0:   # stereo outliers are dropped
                cf.map_points[i] = None
        self.matches_inliers = inliers
        st["inliers"] = inliers
        return inliers >= 30

    # ---- output (src/System.cc:334-486) ---------------------------------------------------------
    def _frame_poses(self):
        """Tcw of every recorded frame, Tcr * Tr(w) with Two of the first keyframe."""
        if not self.keyframes:
            return []
        Two = pose_inverse(sorted(self.keyframes, key=lambda k: k.id)[0].tcw)
        out = []
        for Tcr, kf, t, lost in zip(self.rel_poses, self.references, self.frame_times, self.lost):
            Trw = np.eye(4, dtype=np.float32)
            while kf.bad:   # keyframe culling is out of scope, kept for the reference's shape
                Trw = _mul(Trw, kf.tcp)
                kf = kf.parent
            Trw = _mul(Trw, kf.tcw, Two)
            out.append((_mul(Tcr, Trw), t, lost))
        return out

    def trajectory_twc(self) -> np.ndarray:
        """(n_frames, 4, 4) float32 Twc as SaveTrajectoryKITTI computes them."""
        return np.array([pose_inverse(T) for T, _, _ in self._frame_poses()], np.float32).reshape(-1, 4, 4)

    def SaveTrajectoryKITTI(self, filename: str):
        """System::SaveTrajectoryKITTI (src/System.cc:433-486): 3x4 Twc per frame, fixed, 9 digits."""
        with open(filename, "w") as f:
            for Tcw, _, _ in self._frame_poses():
                Rwc = Tcw[:3, :3].T
                twc = -_mul(Rwc, Tcw[:3, 3:4])[:, 0]
                row = [Rwc[0, 0], Rwc[0, 1], Rwc[0, 2], twc[0], Rwc[1, 0], Rwc[1, 1], Rwc[1, 2], twc[1],
                       Rwc[2, 0], Rwc[2, 1], Rwc[2, 2], twc[2]]
                f.write(" ".join(f"{float(np.float32(v)):.9f}" for v in row) + "\n")

    def SaveTrajectoryTUM(self, filename: str):
        """System::SaveTrajectoryTUM (src/System.cc:334-389): lost frames skipped."""
        with open(filename, "w") as f:
            for Tcw, t, lost in self._frame_poses():
                if lost:
                    continue
                Rwc = Tcw[:3, :3].T
                twc = -_mul(Rwc, Tcw[:3, 3:4])[:, 0]
                q = quaternion_xyzw(Rwc)
                f.write(f"{t:.6f} " + " ".join(f"{float(v):.9f}" for v in (*twc, *q)) + "\n")

    def SaveKeyFrameTrajectoryTUM(self, filename: str):
        """System::SaveKeyFrameTrajectoryTUM (src/System.cc:392-431)."""
        with open(filename, "w") as f:
            for kf in sorted(self.keyframes, key=lambda k: k.id):
                if kf.bad:
                    continue
                q = quaternion_xyzw(kf.tcw[:3, :3].T)
                t = kf.Ow
                f.write(f"{kf.timestamp:.6f} " + " ".join(f"{float(v):.7f}" for v in (*t, *q)) + "\n")

    def Shutdown(self):
        self.backend.close()


def ate_rmse(est_twc: np.ndarray, gt_twc: np.ndarray) -> float:
    """Absolute trajectory error (translation RMSE, metres) of camera centres, both trajectories
    expressed relative to their first frame (the reference's files start at the first keyframe)."""
    est = np.asarray(est_twc, np.float64)
    gt = np.asarray(gt_twc, np.float64)
    g0 = np.linalg.inv(gt[0])
    e0 = np.linalg.inv(est[0])
    d = [(e0 @ e)[:3, 3] - (g0 @ g)[:3, 3] for e, g in zip(est, gt)]
    return float(np.sqrt(np.mean(np.sum(np.square(d), axis=1))))
