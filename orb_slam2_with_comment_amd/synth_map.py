"""Synthetic map state for matcher / BA workloads.

Map points are created the way ORB-SLAM2 creates them from a stereo frame
(Frame::UnprojectStereo, src/Frame.cc:697-712; MapPoint::UpdateNormalAndDepth,
src/MapPoint.cc:339-390): back-projected stereo keypoints with the keypoint's descriptor,
normal = viewing direction, max distance = dist x scale[octave], min = max / scale[L-1].
"""
from __future__ import annotations

import numpy as np

from .types import LFPOINT_DTYPE, LF_HAS_MP, LF_OUTLIER, MAPPOINT_DTYPE, MP_BAD, MP_HAS_OBS, MP_SEEN


def tcw_from_twc(Twc: np.ndarray) -> np.ndarray:
    T = np.eye(4)
    R = Twc[:3, :3]
    T[:3, :3] = R.T
    T[:3, 3] = -R.T @ Twc[:3, 3]
    return T.astype(np.float32)


def unproject(keys, depth, cam, Twc):
    z = depth.astype(np.float64)
    x = (keys["x"] - cam.cx) * z / cam.fx
    y = (keys["y"] - cam.cy) * z / cam.fy
    pc = np.stack([x, y, z], -1)
    return pc @ Twc[:3, :3].T + Twc[:3, 3]


def mappoints_from_frame(keys, desc, depth, cam, Twc, scale_factors, rng=None, bad_frac=0.0, seen_frac=0.0,
                         noobs_frac=0.0):
    ok = depth > 0
    idx = np.nonzero(ok)[0]
    pw = unproject(keys[idx], depth[idx], cam, Twc)
    mp = np.zeros(len(idx), MAPPOINT_DTYPE)
    mp["pos"] = pw.astype(np.float32)
    Ow = Twc[:3, 3]
    d = pw - Ow
    dist = np.linalg.norm(d, axis=1)
    mp["normal"] = (d / dist[:, None]).astype(np.float32)
    sf = np.asarray(scale_factors, np.float32)
    mp["max_distance"] = (dist * sf[keys["octave"][idx]]).astype(np.float32)
    mp["min_distance"] = (mp["max_distance"] / sf[-1]).astype(np.float32)
    mp["desc"] = desc[idx]
    flags = np.full(len(idx), MP_HAS_OBS, np.uint32)
    if rng is not None:
        flags[rng.random(len(idx)) < bad_frac] |= MP_BAD
        flags[rng.random(len(idx)) < seen_frac] |= MP_SEEN
        flags[rng.random(len(idx)) < noobs_frac] &= ~np.uint32(MP_HAS_OBS)
    mp["flags"] = flags
    return mp, idx


def lastframe_points(keys, desc, depth, cam, Twc, rng=None, outlier_frac=0.05, noobs_frac=0.0):
    n = len(keys)
    lf = np.zeros(n, LFPOINT_DTYPE)
    ok = depth > 0
    lf["pos"][ok] = unproject(keys[ok], depth[ok], cam, Twc).astype(np.float32)
    lf["desc"] = desc
    flags = np.where(ok, LF_HAS_MP | MP_HAS_OBS, 0).astype(np.uint32)
    if rng is not None:
        flags[ok & (rng.random(n) < outlier_frac)] |= LF_OUTLIER
        flags[ok & (rng.random(n) < noobs_frac)] &= ~np.uint32(MP_HAS_OBS)
    lf["flags"] = flags
    return lf


# bit positions used to quantise descriptors into synthetic vocabulary nodes
_NODE_BITS = (3, 37, 71, 101, 139, 167, 199, 233)


def bow_nodes(desc: np.ndarray, bits=_NODE_BITS) -> np.ndarray:
    """Synthetic DBoW2 node id per descriptor (the ORB vocabulary is not available offline,
    .MISSING_LARGE_BLOBS:1): descriptors that agree on 8 fixed bits share a node."""
    b = np.unpackbits(np.asarray(desc, np.uint8).reshape(-1, 32), axis=1, bitorder="little")
    node = np.zeros(len(b), np.int64)
    for k, bit in enumerate(bits):
        node |= b[:, bit].astype(np.int64) << k
    return node


def local_ba_problem(seed=42, n_free=20, n_fixed=4, n_points=3000, stereo_frac=0.8, outlier_frac=0.05,
                     obs_min=3, obs_max=8, cam=None, pose_noise=(0.02, 0.1), point_noise=0.2, first_id=10):
    """Config 3 of BASELINE.json / SURVEY.md §8(d): 20 free KFs (1 m spacing, yaw +-0.2 deg) +
    4 fixed observer KFs, 3000 points in x[-10,10] y[-2,2] z[5,40] m ahead, 3-8 observations per
    point (~15k edges), octave from distance (PredictScale), sigma = 1 px x scale, 80 % stereo,
    5 % outliers (+-20 px), initial perturbation +-0.02 rad / +-0.1 m, +-0.2 m on points.
    Returns (BAProblem, ground truth dict)."""
    from . import synth
    from .types import BA_EDGE_DTYPE, BA_KF_DTYPE, BA_PT_DTYPE, BAProblem
    cam = cam or synth.KITTI
    rng = np.random.default_rng(seed)
    sf = np.array([1.2 ** i for i in range(8)], np.float64)
    n_kf = n_free + n_fixed
    Twc = []
    for k in range(n_kf):
        z = float(k - n_fixed)  # fixed observers sit behind the local window
        yaw = np.deg2rad(rng.uniform(-0.2, 0.2) * (k - n_fixed))
        T = np.eye(4)
        T[:3, :3] = [[np.cos(yaw), 0, np.sin(yaw)], [0, 1, 0], [-np.sin(yaw), 0, np.cos(yaw)]]
        T[:3, 3] = [rng.uniform(-0.2, 0.2), rng.uniform(-0.05, 0.05), z]
        Twc.append(T)
    P = np.stack([rng.uniform(-10, 10, n_points), rng.uniform(-2, 2, n_points),
                  rng.uniform(5, 40, n_points) + n_free * 0.5], -1)
    edges, kept_pts = [], []
    for p in range(n_points):
        vis = []
        for k in range(n_kf):
            Tcw = np.linalg.inv(Twc[k])
            pc = Tcw[:3, :3] @ P[p] + Tcw[:3, 3]
            if pc[2] <= 0.5:
                continue
            u = cam.fx * pc[0] / pc[2] + cam.cx
            v = cam.fy * pc[1] / pc[2] + cam.cy
            if 0 <= u < cam.width and 0 <= v < cam.height:
                vis.append((k, u, v, pc[2]))
        if len(vis) < 2:
            continue
        m = min(len(vis), int(rng.integers(obs_min, obs_max + 1)))
        sel = sorted(rng.choice(len(vis), m, replace=False))
        pi = len(kept_pts)
        kept_pts.append(p)
        for s in sel:  # observation map order: by keyframe id
            k, u, v, z = vis[s]
            dist = z
            octave = int(np.clip(np.floor(np.log(max(dist / 8.0, 1.0)) / np.log(1.2)), 0, 7))
            sigma = sf[octave]
            uu = u + rng.normal(0, sigma)
            vv = v + rng.normal(0, sigma)
            ur = -1.0
            if rng.random() < stereo_frac:
                ur = u - cam.bf / z + rng.normal(0, sigma)
            if rng.random() < outlier_frac:
                uu += rng.choice([-20, 20])
                vv += rng.choice([-20, 20])
            edges.append((pi, k, uu, vv, ur, 1.0 / (sigma * sigma)))
    kfs = np.zeros(n_kf, BA_KF_DTYPE)
    for k in range(n_kf):
        T = Twc[k].copy()
        if k >= n_fixed:
            a = rng.uniform(-pose_noise[0], pose_noise[0], 3)
            th = np.linalg.norm(a)
            K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]]) / max(th, 1e-12)
            dR = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
            T[:3, :3] = dR @ T[:3, :3]
            T[:3, 3] += rng.uniform(-pose_noise[1], pose_noise[1], 3)
        kfs[k]["tcw"] = tcw_from_twc(T).reshape(-1)
        kfs[k]["id"] = first_id - n_fixed + k
        kfs[k]["fixed"] = 1 if k < n_fixed else 0
        kfs[k]["fx"], kfs[k]["fy"], kfs[k]["cx"], kfs[k]["cy"], kfs[k]["bf"] = cam.fx, cam.fy, cam.cx, cam.cy, cam.bf
    pts = np.zeros(len(kept_pts), BA_PT_DTYPE)
    pts["pos"] = (P[kept_pts] + rng.uniform(-point_noise, point_noise, (len(kept_pts), 3))).astype(np.float32)
    pts["id"] = 1000 + np.arange(len(kept_pts))
    e = np.array(edges, dtype=[("point", "<i4"), ("kf", "<i4"), ("u", "<f8"), ("v", "<f8"), ("ur", "<f8"),
                               ("inv_sigma2", "<f8")]).astype(BA_EDGE_DTYPE)
    gt = {"Twc": np.stack(Twc), "points": P[kept_pts]}
    return BAProblem(kfs, pts, e), gt


def pose_problem(seed=0, n_obs=600, stereo_frac=0.7, outlier_frac=0.1, cam=None, pose_noise=(0.01, 0.08),
                 nframes=1, point_noise=0.0005):
    """Synthetic Frames for Optimizer::PoseOptimization (src/Optimizer.cc:257-481), the
    TrackWithMotionModel / TrackLocalMap situation: `n_obs` matched map points per frame at
    3-40 m, keypoint noise sigma = 1 px x scale (octave from distance, PredictScale rule), a
    `stereo_frac` share with a right coordinate, `outlier_frac` gross outliers (10-30 px), map
    points off by `point_noise` x depth, and an initial pose off by +-pose_noise (rad, m).
    Returns (frames POSE_FRAME_DTYPE[nframes], obs POSE_OBS_DTYPE[nframes * n_obs], gt Tcw list)."""
    from . import synth
    from .types import POSE_FRAME_DTYPE, POSE_OBS_DTYPE
    cam = cam or synth.KITTI
    rng = np.random.default_rng(seed)
    frames = np.zeros(nframes, POSE_FRAME_DTYPE)
    obs = np.zeros(nframes * n_obs, POSE_OBS_DTYPE)
    gts = []
    for f in range(nframes):
        yaw = rng.uniform(-0.3, 0.3)
        Twc = np.eye(4)
        Twc[:3, :3] = [[np.cos(yaw), 0, np.sin(yaw)], [0, 1, 0], [-np.sin(yaw), 0, np.cos(yaw)]]
        Twc[:3, 3] = rng.uniform(-5, 5, 3)
        Tcw = tcw_from_twc(Twc).astype(np.float64)
        u = rng.uniform(20, cam.width - 20, n_obs)
        v = rng.uniform(20, cam.height - 20, n_obs)
        z = np.exp(rng.uniform(np.log(3.0), np.log(40.0), n_obs))
        Xc = np.stack([(u - cam.cx) * z / cam.fx, (v - cam.cy) * z / cam.fy, z], -1)
        Xw = Xc @ Twc[:3, :3].T + Twc[:3, 3]
        Xw += rng.normal(0, 1, Xw.shape) * (point_noise * z)[:, None]
        octave = np.clip(np.floor(np.log(np.maximum(z / 8.0, 1.0)) / np.log(1.2)), 0, 7).astype(int)
        sigma = 1.2 ** octave
        uu = u + rng.normal(0, 1, n_obs) * sigma
        vv = v + rng.normal(0, 1, n_obs) * sigma
        ur = np.where(rng.random(n_obs) < stereo_frac, u - cam.bf / z + rng.normal(0, 1, n_obs) * sigma, -1.0)
        bad = rng.random(n_obs) < outlier_frac
        du = rng.uniform(10, 30, n_obs) * rng.choice([-1, 1], n_obs)
        dv = rng.uniform(10, 30, n_obs) * rng.choice([-1, 1], n_obs)
        uu = np.where(bad, uu + du, uu)
        vv = np.where(bad, vv + dv, vv)
        ur = np.where(bad & (ur >= 0), ur + du, ur)
        sl = slice(f * n_obs, (f + 1) * n_obs)
        obs["Xw"][sl] = Xw.astype(np.float32)
        obs["u"][sl], obs["v"][sl], obs["ur"][sl] = uu, vv, ur
        obs["inv_sigma2"][sl] = (1.0 / (sigma * sigma)).astype(np.float32)
        obs["index"][sl] = rng.permutation(4 * n_obs)[:n_obs]
        # initial estimate: the motion model's guess, a few cm / mrad off
        a = rng.uniform(-pose_noise[0], pose_noise[0], 3)
        th = np.linalg.norm(a)
        K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]]) / max(th, 1e-12)
        dR = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
        T0 = Tcw.copy()
        T0[:3, :3] = dR @ Tcw[:3, :3]
        T0[:3, 3] += rng.uniform(-pose_noise[1], pose_noise[1], 3)
        frames[f]["tcw"] = T0.astype(np.float32).reshape(-1)
        frames[f]["fx"], frames[f]["fy"], frames[f]["cx"], frames[f]["cy"], frames[f]["bf"] = (
            cam.fx, cam.fy, cam.cx, cam.cy, cam.bf)
        frames[f]["obs_begin"], frames[f]["n_obs"] = f * n_obs, n_obs
        gts.append(Tcw)
    return frames, obs, gts
