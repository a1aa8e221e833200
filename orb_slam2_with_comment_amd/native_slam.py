"""System::TrackStereo on the native host loop (csrc/slam.cpp, orbmi_slam_* in include/orbmi.h):
the map, Tracking and the synchronous LocalMapping in C++ around the MI355X operators, with the
Python interface of system.StereoSLAM (TrackStereo, per-frame stats, trajectory writers) so the
two can be compared frame by frame.  system.StereoSLAM stays the readable form of the same host
logic (and the one the tests also run on the CPU oracle)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._capi import check, lib
from .system import LOST, NO_IMAGES_YET, NOT_INITIALIZED, OK, pose_inverse  # noqa: F401


class SlamSettings(C.Structure):
    """orbmi_slam_settings (include/orbmi.h)."""
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float),
                ("th_depth", C.c_float), ("min_frames", C.c_int), ("max_frames", C.c_int), ("width", C.c_int),
                ("height", C.c_int), ("n_features", C.c_int), ("scale_factor", C.c_float), ("n_levels", C.c_int),
                ("ini_th_fast", C.c_int), ("min_th_fast", C.c_int), ("local_ba", C.c_int), ("local_mapping", C.c_int),
                ("async_local_mapping", C.c_int)]


class FrameStats(C.Structure):
    _fields_ = [(k, C.c_int) for k in ("frame", "n", "state", "init", "track", "lf_matches", "bow_matches",
                                       "nmatches_map", "local_map_points", "local_matches", "inliers", "need_kf",
                                       "keyframes", "mappoints", "reset")]


_TRACK = {1: "motion_model", 2: "reference_kf"}


class NativeStereoSLAM:
    """StereoSLAM with the host loop in C++ (orbmi_slam).  `stats` mirrors system.StereoSLAM.stats:
    one dict per frame with the counters the stage that ran produced."""

    def __init__(self, settings, device: int = 0, vocabulary=None, local_ba: bool = True, local_mapping: bool = True,
                 async_local_mapping: bool = False, record: bool = False):
        """record: keep the schedule, the LocalBA log and the per-keyframe state log
        (orbmi_slam_set_recording) for schedule(), local_ba_log() and keyframe_state_log()."""
        from .settings import Settings, load_settings
        s = settings if isinstance(settings, Settings) else load_settings(settings)
        if s.width <= 0 or s.height <= 0:
            raise ValueError("settings need Camera.width / Camera.height")
        self.settings = s
        self._voc = None
        if vocabulary is not None:
            from .vocabulary import ORBVocabulary
            self._voc = ORBVocabulary(vocabulary, device)
        c = SlamSettings(float(s.fx), float(s.fy), float(s.cx), float(s.cy), float(s.bf), float(s.th_depth),
                         int(s.min_frames), int(s.max_frames), int(s.width), int(s.height), int(s.n_features),
                         float(s.scale_factor), int(s.n_levels), int(s.ini_th_fast), int(s.min_th_fast),
                         1 if local_ba else 0, 1 if local_mapping else 0, 1 if async_local_mapping else 0)
        h = C.c_void_p()
        check("orbmi_slam_create", lib().orbmi_slam_create(C.addressof(c), device,
                                                           self._voc._h if self._voc else None, C.byref(h)))
        self._h = h
        self._tcw = np.zeros(16, np.float32)
        if record:
            check("orbmi_slam_set_recording", lib().orbmi_slam_set_recording(h, 1))

    def TrackStereo(self, imLeft, imRight, timestamp: float, next_pair=None):
        """System::TrackStereo.  next_pair = (imLeft, imRight) of the next call: its Frame
        constructor (extraction + stereo) then runs on the GPU while this frame is tracked
        (orbmi_slam_track_stereo_ahead); the next call must pass those same arrays."""
        L = np.ascontiguousarray(imLeft, np.uint8)
        R = np.ascontiguousarray(imRight, np.uint8)
        if L.shape != R.shape or L.ndim != 2:
            raise ValueError("TrackStereo expects two gray images of the same size")
        has = C.c_int()
        if next_pair is None and not getattr(self, "_ahead", None):
            check("orbmi_slam_track_stereo", lib().orbmi_slam_track_stereo(
                self._h, L.ctypes.data, R.ctypes.data, L.shape[0], L.shape[1], L.strides[0], float(timestamp),
                self._tcw.ctypes.data, C.byref(has)))
        else:
            nL = nR = None
            if next_pair is not None:
                nL = np.ascontiguousarray(next_pair[0], np.uint8)
                nR = np.ascontiguousarray(next_pair[1], np.uint8)
                if nL.shape != L.shape or nR.shape != L.shape:
                    raise ValueError("next_pair must have the geometry of this pair")
            check("orbmi_slam_track_stereo_ahead", lib().orbmi_slam_track_stereo_ahead(
                self._h, L.ctypes.data, R.ctypes.data, L.shape[0], L.shape[1], L.strides[0], float(timestamp),
                None if nL is None else nL.ctypes.data, None if nR is None else nR.ctypes.data,
                self._tcw.ctypes.data, C.byref(has)))
            self._ahead = (nL, nR) if nL is not None else None  # the buffers stay alive until used
        return self._tcw.reshape(4, 4).copy() if has.value else None

    def counts(self):
        f, k, m, b = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        check("orbmi_slam_get_counts", lib().orbmi_slam_get_counts(self._h, C.byref(f), C.byref(k), C.byref(m),
                                                                   C.byref(b)))
        return {"frames": f.value, "keyframes": k.value, "mappoints": m.value, "local_ba_calls": b.value}

    @property
    def stats(self) -> list:
        out = []
        f = 0
        while True:  # one record per TrackStereo call (frame ids restart after a reset)
            st = FrameStats()
            if lib().orbmi_slam_get_stats(self._h, f, C.byref(st)) != 0:
                break
            f += 1
            d = {k: getattr(st, k) for k, _ in FrameStats._fields_}
            d = {k: v for k, v in d.items() if v != -1}
            if "track" in d:
                d["track"] = _TRACK.get(d["track"], d["track"])
            if "init" in d:
                d["init"] = bool(d["init"])
            if "need_kf" in d:
                d["need_kf"] = bool(d["need_kf"])
            out.append(d)
        return out

    def frame_poses(self):
        """(Tcw [n, 4, 4], timestamps, lost) as SaveTrajectoryKITTI / TUM compute them."""
        n = C.c_int()
        cap = max(self.counts()["frames"], 1)
        T = np.zeros((cap, 16), np.float32)
        ts = np.zeros(cap, np.float64)
        lost = np.zeros(cap, np.uint8)
        check("orbmi_slam_get_trajectory", lib().orbmi_slam_get_trajectory(self._h, T.ctypes.data, ts.ctypes.data,
                                                                           lost.ctypes.data, cap, C.byref(n)))
        k = n.value
        return T[:k].reshape(-1, 4, 4), ts[:k], lost[:k].astype(bool)

    def trajectory_twc(self) -> np.ndarray:
        T, _, _ = self.frame_poses()
        return np.array([pose_inverse(t) for t in T], np.float32).reshape(-1, 4, 4)

    def SaveTrajectoryKITTI(self, filename: str):
        check("orbmi_slam_save_trajectory_kitti", lib().orbmi_slam_save_trajectory_kitti(self._h, filename.encode()))

    def SaveTrajectoryTUM(self, filename: str):
        check("orbmi_slam_save_trajectory_tum", lib().orbmi_slam_save_trajectory_tum(self._h, filename.encode()))

    def SaveKeyFrameTrajectoryTUM(self, filename: str):
        check("orbmi_slam_save_keyframe_trajectory_tum",
              lib().orbmi_slam_save_keyframe_trajectory_tum(self._h, filename.encode()))

    PHASES = ("frame_ctor", "map_lock_wait", "lf_search", "lf_pose", "local_kf_points", "local_records",
              "frustum", "local_search", "local_pose", "keyframe", "total", "lm_process", "lm_point_culling",
              "lm_create_points", "lm_search_in_neighbors", "lm_local_ba", "lm_keyframe_culling", "lm_total",
              "lm_create_points_call", "lm_fuse_search_calls", "lm_distinctive_calls",
              "lm_lock_wait", "lm_sin_prep", "lm_sin_redo_check", "lm_sin_replay", "lm_normals", "lm_connections",
              "lm_obs_rows", "lm_ba_gather", "lm_ba_call", "lm_ba_writeback")

    def phase_ms(self):
        """Mean wall ms per tracked frame of each phase of TrackStereo (orbmi_slam_get_phase_ms)."""
        ms = np.zeros(len(self.PHASES))
        n = C.c_long()
        check("orbmi_slam_get_phase_ms", lib().orbmi_slam_get_phase_ms(self._h, ms.ctypes.data, len(ms), C.byref(n)))
        return {k: round(float(v) / max(n.value, 1), 4) for k, v in zip(self.PHASES, ms)}

    def schedule(self) -> np.ndarray:
        """The concurrent run's schedule (orbmi_slam_get_schedule): int32 [n, 3] rows of (thread,
        label, arg), one per acquisition of the map lock, in order (empty when synchronous)."""
        return self._records("orbmi_slam_get_schedule", 3)

    def local_ba_log(self) -> np.ndarray:
        """Per LocalBundleAdjustment call: int32 rows of (keyframe, stop_check, aborted, checks,
        iterations0, iterations1, edges, erased) (orbmi_slam_get_local_ba_log)."""
        return self._records("orbmi_slam_get_local_ba_log", 8)

    def local_mapping_counts(self) -> dict:
        """LocalMapping::Run outcomes (orbmi_slam_get_local_mapping_counts)."""
        v = np.zeros(5, np.int32)
        check("orbmi_slam_get_local_mapping_counts",
              lib().orbmi_slam_get_local_mapping_counts(self._h, v.ctypes.data, len(v)))
        return dict(zip(("jobs", "search_in_neighbors_skipped", "ba_skipped", "ba_interrupted", "ba_aborted"),
                        (int(x) for x in v)))

    def keyframe_state_log(self) -> np.ndarray:
        """Per keyframe and LocalMapping stage: int32 rows of (keyframe, stage, schedule event, a,
        b, c) (orbmi_slam_get_keyframe_state_log; include/orbmi_debug.h ORBMI_KF_STATE_*)."""
        return self._records("orbmi_slam_get_keyframe_state_log", 6)

    def _records(self, fn, width):
        n = C.c_int()
        rc = getattr(lib(), fn)(self._h, None, 0, C.byref(n))
        out = np.zeros((max(n.value, 1), width), np.int32)
        if n.value:
            check(fn, getattr(lib(), fn)(self._h, out.ctypes.data, n.value, C.byref(n)))
        elif rc not in (0,):
            check(fn, rc)
        return out[:n.value]

    def WaitLocalMapping(self):
        """Block until the mapping thread has processed every queued keyframe (async mode)."""
        check("orbmi_slam_wait_local_mapping", lib().orbmi_slam_wait_local_mapping(self._h))

    def Shutdown(self):
        if getattr(self, "_h", None):
            lib().orbmi_slam_destroy(self._h)
            self._h = None
        if self._voc is not None:
            self._voc.close()
            self._voc = None

    def __del__(self):
        try:
            self.Shutdown()
        except Exception:
            pass
