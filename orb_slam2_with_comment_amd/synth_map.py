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
