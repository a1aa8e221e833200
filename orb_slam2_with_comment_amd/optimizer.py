"""Python mirror of Optimizer::LocalBundleAdjustment (include/Optimizer.h:62) over the C ABI.

`gather_local_ba` restates the graph assembly of src/Optimizer.cc:486-683 (local keyframes =
pKF + covisible, local points, fixed observer keyframes, one edge per observation) over a
minimal map model; `LocalBA.run` optimises the assembled graph on the GPU."""
from __future__ import annotations

import ctypes as C
import dataclasses

import numpy as np

from ._capi import check, lib
from .types import BA_EDGE_DTYPE, BA_KF_DTYPE, BA_PT_DTYPE, BAProblem


class LocalBA:
    def __init__(self, device: int = 0):
        h = C.c_void_p()
        check("orbmi_ba_create", lib().orbmi_ba_create(device, C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().orbmi_ba_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stop_at_check(self, k: int):
        """The deterministic pbStopFlag (orbmi_ba_set_stop_at_check): later calls read the flag
        raised from their k-th check on; k < 0 turns it off."""
        check("orbmi_ba_set_stop_at_check", lib().orbmi_ba_set_stop_at_check(self._h, int(k)))

    def run(self, problem: BAProblem, stop: C.c_int | None = None, stop_at_check: int | None = None):
        if stop_at_check is not None:
            self.set_stop_at_check(stop_at_check)
        r, tcw, pos, erase = problem.result_buffers()
        v = problem.view()
        check("orbmi_local_bundle_adjustment",
              lib().orbmi_local_bundle_adjustment(self._h, C.addressof(v), C.addressof(r),
                                                  C.addressof(stop) if stop is not None else None))
        n = len(problem.kfs), len(problem.pts), len(problem.edges)
        return {"tcw": tcw[:n[0]].reshape(-1, 4, 4), "pos": pos[:n[1]], "erase": erase[:n[2]].astype(bool),
                "iterations": tuple(r.iterations), "chi2": tuple(r.chi2), "aborted": r.aborted,
                "stop_check": r.stop_check, "checks": r.checks}


class PoseOptimizer:
    """Optimizer::PoseOptimization(Frame*) (include/Optimizer.h:58) on the GPU, batched: one
    workgroup per frame.  `run(frames, obs)` updates the POSE_FRAME_DTYPE records in place
    (tcw, inliers = the reference's return value, iterations) and returns mvbOutlier per obs."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        check("orbmi_pose_create", lib().orbmi_pose_create(device, C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().orbmi_pose_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run(self, frames: np.ndarray, obs: np.ndarray) -> np.ndarray:
        from .types import POSE_FRAME_DTYPE, POSE_OBS_DTYPE
        assert frames.dtype == POSE_FRAME_DTYPE and obs.dtype == POSE_OBS_DTYPE
        assert frames.flags.c_contiguous and obs.flags.c_contiguous
        out = np.zeros(len(obs), np.uint8)
        check("orbmi_pose_optimization",
              lib().orbmi_pose_optimization(self._h, frames.ctypes.data, len(frames), obs.ctypes.data, len(obs),
                                            out.ctypes.data))
        return out.astype(bool)

    def run_device(self, frames_ptr: int, nframes: int, obs_ptr: int, nobs: int, outlier_ptr: int):
        """Device-resident frames / observations / flags: enqueued on the handle's stream."""
        check("orbmi_pose_optimization",
              lib().orbmi_pose_optimization(self._h, frames_ptr, nframes, obs_ptr, nobs, outlier_ptr))

    def synchronize(self):
        check("orbmi_pose_synchronize", lib().orbmi_pose_synchronize(self._h))

    def share_stream(self, extractor_handle):
        check("orbmi_pose_share_stream", lib().orbmi_pose_share_stream(self._h, extractor_handle))

    def PoseOptimization(self, view, inv_level_sigma2: np.ndarray, mappoints, rec, outlier):
        """Optimizer::PoseOptimization(Frame*) with its edge assembly: `view` = FrameView
        (initial tcw), `mappoints` = FrameMapPoints, rec = POSE_FRAME_DTYPE record (numpy, or a
        device address), outlier = per-keypoint mvbOutlier (numpy u8, or a device address).
        Returns the inlier count for host records, None when enqueued on the device."""
        sig = np.ascontiguousarray(inv_level_sigma2, np.float32)
        host = isinstance(rec, np.ndarray)
        rp = rec.ctypes.data if host else rec
        op = outlier.ctypes.data if isinstance(outlier, np.ndarray) else outlier
        check("orbmi_pose_optimization_frame",
              lib().orbmi_pose_optimization_frame(self._h, C.addressof(view), sig.ctypes.data, C.addressof(mappoints),
                                                  rp, op))
        return int(np.asarray(rec["inliers"]).reshape(-1)[0]) if host else None

    def PoseOptimizationTrack(self, view, inv_level_sigma2: np.ndarray, mappoints, rec: int, outlier: int, stage: int,
                              occupied_out, counts: int):
        """PoseOptimization followed by Tracking's pass over mvpMapPoints (orbmi_track_update_matches
        `stage`: 0 = TrackWithMotionModel's outlier discard, 1 = TrackLocalMap's statistics) in one
        launch; every address is device memory, enqueued on the handle's stream."""
        sig = np.ascontiguousarray(inv_level_sigma2, np.float32)
        check("orbmi_pose_optimization_frame_track",
              lib().orbmi_pose_optimization_frame_track(self._h, C.addressof(view), sig.ctypes.data,
                                                        C.addressof(mappoints), rec, outlier, int(stage),
                                                        occupied_out, counts))


# ---- minimal map model for the graph assembly (src/Optimizer.cc:486-534) ------------------
@dataclasses.dataclass(eq=False)
class KeyFrame:
    id: int
    tcw: np.ndarray                     # 4x4 float32
    keys_un: np.ndarray                 # KP_DTYPE
    u_right: np.ndarray                 # float32 (-1 = mono)
    inv_level_sigma2: np.ndarray        # mvInvLevelSigma2
    cam: object
    map_points: list = dataclasses.field(default_factory=list)   # MapPoint or None per keypoint
    covisible: list = dataclasses.field(default_factory=list)    # GetVectorCovisibleKeyFrames order
    bad: bool = False


@dataclasses.dataclass(eq=False)
class MapPoint:
    id: int
    pos: np.ndarray
    observations: dict = dataclasses.field(default_factory=dict)  # KeyFrame -> keypoint index
    bad: bool = False


def gather_local_ba(pKF: KeyFrame):
    """Assemble the LocalBundleAdjustment graph around pKF exactly like the reference
    (local KFs, local MPs in first-seen order, fixed cameras, edges per observation in KF-id
    order -- the build's deterministic replacement of std::map<KeyFrame*> pointer order)."""
    local_kfs = [pKF] + [k for k in pKF.covisible if not k.bad]
    local_set = {id(k) for k in [pKF] + pKF.covisible}
    local_mps, seen = [], set()
    for kf in local_kfs:
        for mp in kf.map_points:
            if mp is not None and not mp.bad and id(mp) not in seen:
                seen.add(id(mp))
                local_mps.append(mp)
    fixed, fixed_set = [], set()
    for mp in local_mps:
        for kf in sorted(mp.observations, key=lambda k: k.id):
            if id(kf) not in local_set and id(kf) not in fixed_set:
                fixed_set.add(id(kf))
                if not kf.bad:
                    fixed.append(kf)
    kfs = local_kfs + fixed
    kidx = {id(k): i for i, k in enumerate(kfs)}
    K = np.zeros(len(kfs), BA_KF_DTYPE)
    for i, k in enumerate(kfs):
        K[i]["tcw"] = np.asarray(k.tcw, np.float32).reshape(-1)
        K[i]["id"] = k.id
        K[i]["fixed"] = 1 if (i >= len(local_kfs) or k.id == 0) else 0
        K[i]["fx"], K[i]["fy"], K[i]["cx"], K[i]["cy"], K[i]["bf"] = k.cam.fx, k.cam.fy, k.cam.cx, k.cam.cy, k.cam.bf
    P = np.zeros(len(local_mps), BA_PT_DTYPE)
    if local_mps:
        P["pos"] = np.array([mp.pos for mp in local_mps], np.float32)
        P["id"] = [mp.id for mp in local_mps]
        P["bad"] = [int(mp.bad) for mp in local_mps]
    e_pt, e_kf, e_kp = [], [], []
    for pi, mp in enumerate(local_mps):
        for kf in sorted(mp.observations, key=lambda k: k.id):
            ki = kidx.get(id(kf))
            if kf.bad or ki is None:
                continue
            e_pt.append(pi)
            e_kf.append(ki)
            e_kp.append(mp.observations[kf])
    E = np.zeros(len(e_pt), BA_EDGE_DTYPE)
    if e_pt:
        E["point"], E["kf"] = e_pt, e_kf
        e_kf, e_kp = np.asarray(e_kf), np.asarray(e_kp)
        for ki in np.unique(e_kf):   # one gather per keyframe
            sel = e_kf == ki
            k, j = kfs[ki], e_kp[sel]
            kp = k.keys_un[j]
            E["u"][sel] = kp["x"]
            E["v"][sel] = kp["y"]
            E["ur"][sel] = np.asarray(k.u_right, np.float32)[j]
            E[E.dtype.names[5]][sel] = np.asarray(k.inv_level_sigma2, np.float32)[kp["octave"]]
    return BAProblem(K, P, E), kfs, local_mps
