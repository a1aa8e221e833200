"""Synthetic KITTI- / EuRoC-shaped input.

KITTI-00 and EuRoC are not available offline, so every benchmark and parity test runs on
ray-cast textured planes with exact ground truth: a ground plane at y=+1.65 m, side walls at
x=+-8 m, a canopy at y=-4 m and a far wall, camera moving forward 1 m/frame with 0.2 deg/frame
yaw.  Intrinsics come from the reference's own settings files
(Examples/Stereo/KITTI00-02.yaml, Examples/Monocular/EuRoC.yaml).  The texture is a blocky
multi-scale hash pattern on a smooth gradient plus +-4 uniform noise, seeded per frame, which
gives FAST corners at every pyramid level.
"""
from __future__ import annotations

import dataclasses

import numpy as np


@dataclasses.dataclass(frozen=True)
class Camera:
    width: int
    height: int
    fx: float
    fy: float
    cx: float
    cy: float
    bf: float  # stereo baseline x fx

    @property
    def baseline(self) -> float:
        return self.bf / self.fx


# Examples/Stereo/KITTI00-02.yaml
KITTI = Camera(1241, 376, 718.856, 718.856, 607.1928, 185.2157, 386.1448)
# Examples/Monocular/EuRoC.yaml (bf from Examples/Stereo/EuRoC.yaml)
EUROC = Camera(752, 480, 458.654, 457.296, 367.215, 248.375, 47.90639384423901)

_PLANES = (  # (axis, offset): plane axis == offset in world coordinates
    (1, 1.65),    # ground
    (1, -4.0),    # canopy
    (0, -8.0),    # left wall
    (0, 8.0),     # right wall
    (2, 400.0),   # far wall
)


def _hash01(i: np.ndarray, j: np.ndarray, salt: int) -> np.ndarray:
    h = (i.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)) ^ \
        (j.astype(np.uint64) * np.uint64(0xC2B2AE3D27D4EB4F)) ^ np.uint64(salt * 0x165667B19E3779F9 & (2**64 - 1))
    h ^= h >> np.uint64(29)
    h *= np.uint64(0xBF58476D1CE4E5B9)
    h ^= h >> np.uint64(32)
    return (h >> np.uint64(40)).astype(np.float64) / float(1 << 24)


def pose(frame: int, step: float = 1.0, yaw_deg: float = 0.2) -> np.ndarray:
    """Twc (4x4 float64) of the left camera at `frame`."""
    a = np.deg2rad(yaw_deg * frame)
    T = np.eye(4)
    T[:3, :3] = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
    T[2, 3] = step * frame
    return T


def render(cam: Camera, Twc: np.ndarray, seed: int, noise: float = 4.0,
           return_depth: bool = False):
    """Ray-cast one u8 image (H x W) from camera pose Twc."""
    u = np.arange(cam.width, dtype=np.float64)
    v = np.arange(cam.height, dtype=np.float64)
    uu, vv = np.meshgrid(u, v)
    dc = np.stack([(uu - cam.cx) / cam.fx, (vv - cam.cy) / cam.fy, np.ones_like(uu)], -1)
    dw = dc @ Twc[:3, :3].T
    o = Twc[:3, 3]
    best_t = np.full(uu.shape, np.inf)
    img = np.zeros(uu.shape)
    for pid, (axis, off) in enumerate(_PLANES):
        with np.errstate(divide="ignore", invalid="ignore"):
            t = (off - o[axis]) / dw[..., axis]
        hit = (t > 0) & (t < best_t)
        if not hit.any():
            continue
        p = o + dw[hit] * t[hit][:, None]
        ax = [k for k in range(3) if k != axis]
        a, b = p[:, ax[0]], p[:, ax[1]]
        val = 128.0 + 50.0 * np.sin(0.11 * a + pid) * np.cos(0.07 * b)
        val += 80.0 * (_hash01(np.floor(a / 0.6), np.floor(b / 0.6), 11 + pid) - 0.5)
        val += 50.0 * (_hash01(np.floor(a / 0.17), np.floor(b / 0.17), 23 + pid) - 0.5)
        img[hit] = val
        best_t[hit] = t[hit]
    rng = np.random.default_rng(seed)
    img += rng.uniform(-noise, noise, img.shape)
    out = np.clip(np.rint(img), 0, 255).astype(np.uint8)
    if return_depth:
        return out, best_t  # t along dc (z=1) is the depth
    return out


def stereo_pair(cam: Camera, frame: int, seed_base: int = 1000):
    """(left, right, Twc_left) for frame `frame` of the KITTI-shaped sequence."""
    T = pose(frame)
    TR = T.copy()
    TR[:3, 3] = T[:3, 3] + T[:3, :3] @ np.array([cam.baseline, 0.0, 0.0])
    seed = seed_base + frame
    return render(cam, T, seed), render(cam, TR, seed + 7919), T


def mono(cam: Camera, frame: int, seed_base: int = 5000):
    return render(cam, pose(frame, step=0.05, yaw_deg=0.5), seed_base + frame)
