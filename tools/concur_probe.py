"""Concurrent-LocalMapping diagnostics (tests/test_native_slam_gpu.py's sequence): the native
loop with LocalMapping on its own thread, on the device-resident tracking path and on the staged
one (ORBMI_SLAM_STAGED=1), per-frame tracking statistics and position errors side by side.
python tools/concur_probe.py [runs] [frame period ms: paced as stereo_kitti.cc:95-107, 0 = back to back]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import tempfile  # noqa: E402
import time  # noqa: E402

import numpy as np  # noqa: E402

from orb_slam2_with_comment_amd.native_slam import NativeStereoSLAM  # noqa: E402
from orb_slam2_with_comment_amd.system import ate_rmse  # noqa: E402
from slam_backends import render_sequence, sequence_settings, small_vocabulary  # noqa: E402

KEYS = ("track", "lf_matches", "nmatches_map", "local_map_points", "local_matches", "inliers", "need_kf")


def run(frames, s, voc, staged, period):
    if staged:
        os.environ["ORBMI_SLAM_STAGED"] = "1"
    else:
        os.environ.pop("ORBMI_SLAM_STAGED", None)
    slam = NativeStereoSLAM(s, device=0, vocabulary=voc, async_local_mapping=True)
    t0 = time.perf_counter()
    for f, (L, R, _) in enumerate(frames):
        slam.TrackStereo(L, R, 0.1 * f)
        wait = t0 + (f + 1) * period - time.perf_counter()
        if wait > 0:
            time.sleep(wait)
    slam.WaitLocalMapping()
    T = slam.trajectory_twc()
    st = slam.stats
    c = slam.counts()
    slam.Shutdown()
    return T, st, c


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    period = (float(sys.argv[2]) if len(sys.argv) > 2 else 0.0) * 1e-3
    n = 200
    frames = render_sequence(n)
    gt = np.array([fr[2] for fr in frames])
    voc = small_vocabulary()
    with tempfile.TemporaryDirectory() as d:
        s = sequence_settings(__import__("pathlib").Path(d))
        for r in range(runs):
            for staged in (False, True):
                T, st, c = run(frames, s, voc, staged, period)
                err = np.linalg.norm(T[:, :3, 3] - gt[:, :3, 3], axis=1)
                name = ("staged" if staged else "dev") + f" period {period * 1e3:g} ms"
                jump = int(np.argmax(err > 0.5)) if (err > 0.5).any() else -1
                print(f"{name} run {r}: ATE {ate_rmse(T, gt):.4f} m, max err {err.max():.3f} m at frame "
                      f"{int(err.argmax())}, first frame with err > 0.5 m: {jump}, {c}")
                means = {k: float(np.mean([x.get(k, 0) for x in st])) for k in KEYS
                         if all(isinstance(x.get(k, 0), (int, float)) for x in st)}
                print("   means:", {k: round(v, 1) for k, v in means.items()})
                lo = max(0, (jump if jump >= 0 else int(err.argmax())) - 6)
                for f in range(lo, min(n, lo + 10)):
                    print(f"   frame {f}: err {err[f]:.3f}", {k: st[f].get(k) for k in KEYS})
                sys.stdout.flush()


if __name__ == "__main__":
    main()
