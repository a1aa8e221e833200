"""Settings files of the reference (cv::FileStorage YAML, `%YAML:1.0`) and the values
Tracking derives from them (src/Tracking.cc:53-143).

The reference reads its camera / ORB parameters with `cv::FileStorage` (src/Tracking.cc:53,
src/System.cc:51-57).  That format is not plain YAML (the `%YAML:1.0` directive, `Key:value`
without a space, `!!opencv-matrix` nodes), so it is parsed here directly.  A key that is absent
reads as 0, as `(float)fSettings["missing"]` does in OpenCV; every derived value follows the
float32 arithmetic of the Tracking constructor.
"""
from __future__ import annotations

import dataclasses
import re

import numpy as np

_KEY = re.compile(r"^([A-Za-z_][A-Za-z0-9_.]*)\s*:\s*(.*?)\s*$")


def _scalar(text: str):
    t = text.strip()
    if t.startswith('"') and t.endswith('"') and len(t) >= 2:
        return t[1:-1]
    try:
        return int(t)
    except ValueError:
        pass
    try:
        return float(t)
    except ValueError:
        return t


def read_file_storage(path: str) -> dict:
    """Parse an OpenCV FileStorage YAML file into {key: int | float | str | ndarray}.
    `!!opencv-matrix` nodes (rows / cols / dt / data, possibly spanning lines) become float64
    arrays of shape (rows, cols)."""
    with open(path, "r") as f:
        lines = f.read().splitlines()
    if not lines or not lines[0].startswith("%YAML"):
        raise ValueError(f"{path}: not an OpenCV FileStorage YAML file (missing %YAML header)")
    out: dict = {}
    i = 1
    while i < len(lines):
        raw = lines[i]
        i += 1
        s = raw.split("#", 1)[0].rstrip() if not raw.lstrip().startswith('"') else raw.rstrip()
        if not s.strip() or s.strip() == "---" or raw[:1].isspace():
            continue
        m = _KEY.match(s)
        if not m:
            raise ValueError(f"{path}:{i}: cannot parse {raw!r}")
        key, val = m.group(1), m.group(2)
        if val.startswith("!!opencv-matrix"):
            node, data = {}, None
            while i < len(lines) and (lines[i][:1].isspace() or not lines[i].strip()):
                t = lines[i].split("#", 1)[0].strip()
                i += 1
                if not t:
                    continue
                mm = _KEY.match(t)
                if mm and mm.group(1) != "data":
                    node[mm.group(1)] = _scalar(mm.group(2))
                    continue
                body = t.split(":", 1)[1] if t.startswith("data") else t
                data = (data or "") + body
                if "]" in body:
                    break
            vals = [float(v) for v in data.replace("[", " ").replace("]", " ").replace(",", " ").split()]
            out[key] = np.array(vals, np.float64).reshape(int(node["rows"]), int(node["cols"]))
        else:
            out[key] = _scalar(val)
    return out


def _f32(x) -> np.float32:
    return np.float32(x if isinstance(x, (int, float, np.floating, np.integer)) else 0.0)


@dataclasses.dataclass
class Settings:
    """The Tracking constructor's view of a settings file (src/Tracking.cc:53-143)."""
    fx: np.float32
    fy: np.float32
    cx: np.float32
    cy: np.float32
    K: np.ndarray            # mK, 3x3 float32
    dist_coef: np.ndarray    # mDistCoef: k1 k2 p1 p2 [k3 when k3 != 0], float32
    bf: np.float32           # mbf
    fps: np.float32          # 30 when the file says 0
    min_frames: int          # mMinFrames
    max_frames: int          # mMaxFrames = (int) fps
    rgb: bool                # mbRGB
    n_features: int
    scale_factor: np.float32
    n_levels: int
    ini_th_fast: int
    min_th_fast: int
    th_depth: np.float32     # mThDepth = mbf * (float)ThDepth / fx (stereo / RGB-D)
    depth_map_factor: np.float32
    width: int               # Camera.width / height (read by the examples, not by Tracking)
    height: int
    raw: dict

    @property
    def camera(self):
        """synth.Camera with these intrinsics (what the GPU frame views take)."""
        from .synth import Camera
        return Camera(int(self.width), int(self.height), float(self.fx), float(self.fy), float(self.cx),
                      float(self.cy), float(self.bf))


def load_settings(path: str) -> Settings:
    """Tracking::Tracking's reads of `strSettingPath` (src/Tracking.cc:53-143)."""
    fs = read_file_storage(path)
    g = lambda k: fs.get(k, 0)  # noqa: E731  (cv::FileNode of a missing key reads as 0)
    fx, fy, cx, cy = _f32(g("Camera.fx")), _f32(g("Camera.fy")), _f32(g("Camera.cx")), _f32(g("Camera.cy"))
    K = np.eye(3, dtype=np.float32)
    K[0, 0], K[1, 1], K[0, 2], K[1, 2] = fx, fy, cx, cy
    dist = [_f32(g("Camera.k1")), _f32(g("Camera.k2")), _f32(g("Camera.p1")), _f32(g("Camera.p2"))]
    k3 = _f32(g("Camera.k3"))
    if k3 != 0:
        dist.append(k3)
    fps = _f32(g("Camera.fps"))
    if fps == 0:
        fps = np.float32(30)
    bf = _f32(g("Camera.bf"))
    th_depth = np.float32(np.float32(bf * _f32(g("ThDepth"))) / fx) if fx != 0 else np.float32(0)
    dmf = _f32(g("DepthMapFactor"))
    dmf = np.float32(1) if abs(dmf) < 1e-5 else np.float32(np.float32(1.0) / dmf)
    return Settings(fx=fx, fy=fy, cx=cx, cy=cy, K=K, dist_coef=np.array(dist, np.float32), bf=bf, fps=fps,
                    min_frames=0, max_frames=int(fps), rgb=bool(int(g("Camera.RGB"))),
                    n_features=int(g("ORBextractor.nFeatures")), scale_factor=_f32(g("ORBextractor.scaleFactor")),
                    n_levels=int(g("ORBextractor.nLevels")), ini_th_fast=int(g("ORBextractor.iniThFAST")),
                    min_th_fast=int(g("ORBextractor.minThFAST")), th_depth=th_depth, depth_map_factor=dmf,
                    width=int(g("Camera.width")), height=int(g("Camera.height")), raw=fs)


def write_settings(path: str, cam, n_features=2000, scale_factor=1.2, n_levels=8, ini_th=20, min_th=7,
                   fps=10.0, th_depth=35, rgb=1) -> None:
    """Write a stereo settings file in the reference's format for a synth.Camera (the synthetic
    KITTI-/EuRoC-shaped sequences have no settings file of their own)."""
    rows = [("Camera.fx", cam.fx), ("Camera.fy", cam.fy), ("Camera.cx", cam.cx), ("Camera.cy", cam.cy),
            ("Camera.k1", 0.0), ("Camera.k2", 0.0), ("Camera.p1", 0.0), ("Camera.p2", 0.0),
            ("Camera.width", cam.width), ("Camera.height", cam.height), ("Camera.fps", float(fps)),
            ("Camera.bf", cam.bf), ("Camera.RGB", int(rgb)), ("ThDepth", th_depth),
            ("ORBextractor.nFeatures", int(n_features)), ("ORBextractor.scaleFactor", float(scale_factor)),
            ("ORBextractor.nLevels", int(n_levels)), ("ORBextractor.iniThFAST", int(ini_th)),
            ("ORBextractor.minThFAST", int(min_th))]
    with open(path, "w") as f:
        f.write("%YAML:1.0\n\n")
        for k, v in rows:
            f.write(f"{k}: {v!r}\n" if isinstance(v, float) else f"{k}: {v}\n")
