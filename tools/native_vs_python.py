"""Development check: the native host loop (orbmi_slam) against system.StereoSLAM on the GPU
backend and (optionally) on the oracle backend, frame by frame.  Usage:
python tools/native_vs_python.py N [oracle]"""
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401

from orb_slam2_with_comment_amd import synth  # noqa: E402
from orb_slam2_with_comment_amd.native_slam import NativeStereoSLAM  # noqa: E402
from orb_slam2_with_comment_amd.system import StereoSLAM, ate_rmse  # noqa: E402
from slam_backends import OracleBackend, render_sequence, sequence_settings, small_vocabulary  # noqa: E402

KEYS = ("n", "init", "track", "bow_matches", "lf_matches", "nmatches_map", "local_map_points", "local_matches",
        "inliers", "need_kf", "state", "keyframes", "mappoints")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
use_oracle = len(sys.argv) > 2
t = time.perf_counter()
frames = render_sequence(n)
print(f"rendered {n} frames in {time.perf_counter() - t:.1f} s", flush=True)
s = sequence_settings(tempfile.mkdtemp())
voc = small_vocabulary()
runs = {}
for name in ["native", "python"] + (["oracle"] if use_oracle else []):
    if name == "native":
        slam = NativeStereoSLAM(s, device=0, vocabulary=voc)
    elif name == "python":
        slam = StereoSLAM(s, device=0, vocabulary=voc)
    else:
        slam = StereoSLAM(s, backend=OracleBackend(s, voc))
    t = time.perf_counter()
    times = []
    for f in range(n):
        L, R, _ = frames[f]
        t0 = time.perf_counter()
        slam.TrackStereo(L, R, 0.1 * f)
        times.append(time.perf_counter() - t0)
    el = time.perf_counter() - t
    tw = slam.trajectory_twc()
    gt = np.array([fr[2] for fr in frames])
    ts = np.array(times[10:]) * 1e3
    print(f"{name}: {n / el:.1f} frames/s, median {np.median(ts):.2f} ms, mean {np.mean(ts):.2f} ms after 10, "
          f"ATE {ate_rmse(tw, gt):.4f} m", flush=True)
    runs[name] = (slam.stats, tw)
    slam.Shutdown()
ref_stats, ref_tw = runs["native"]
for name in runs:
    if name == "native":
        continue
    st, tw = runs[name]
    bad = [f for f, (a, b) in enumerate(zip(ref_stats, st)) if {k: a.get(k) for k in KEYS} != {k: b.get(k) for k in KEYS}]
    print(f"native vs {name}: {len(bad)} frames with different decisions; first: {bad[:5]}")
    if bad:
        f = bad[0]
        print("  native:", {k: ref_stats[f].get(k) for k in KEYS})
        print("  " + name + ":", {k: st[f].get(k) for k in KEYS})
    k = min(len(tw), len(ref_tw))
    print(f"  max |dt| {np.abs(tw[:k, :3, 3] - ref_tw[:k, :3, 3]).max():.2e} m, max |dR| "
          f"{np.abs(tw[:k, :3, :3] - ref_tw[:k, :3, :3]).max():.2e}")
