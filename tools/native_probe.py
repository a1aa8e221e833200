"""The native stereo loop (orbmi_slam) over the rendered sequence, synchronous or with the
concurrent LocalMapping, printing the per-phase split -- a target for rocprofv3.
python tools/native_probe.py [frames] [async]"""
import os
import sys
import tempfile
import time

# as bench.py: 8 hardware queues (the process's streams then map onto queues of their own)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from orb_slam2_with_comment_amd.native_slam import NativeStereoSLAM  # noqa: E402
from orb_slam2_with_comment_amd.settings import load_settings, write_settings  # noqa: E402
from orb_slam2_with_comment_amd.synth import KITTI  # noqa: E402
from orb_slam2_with_comment_amd.vocabulary import Vocabulary  # noqa: E402
from slam_backends import render_sequence  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    async_lm = len(sys.argv) > 2 and sys.argv[2] == "async"
    frames = render_sequence(n)
    path = os.path.join(tempfile.mkdtemp(), "KITTI_synth.yaml")
    write_settings(path, KITTI, n_features=2000)
    slam = NativeStereoSLAM(load_settings(path), device=0, vocabulary=Vocabulary.synthetic(k=10, L=5, seed=3),
                            async_local_mapping=async_lm)
    t0 = time.perf_counter()
    for f, (L, R, _) in enumerate(frames):  # the next pair handed over ahead, as bench --mode system
        slam.TrackStereo(L, R, 0.1 * f, next_pair=frames[f + 1][:2] if f + 1 < n else None)
    slam.WaitLocalMapping()
    dt = time.perf_counter() - t0
    c = slam.counts()
    ph = slam.phase_ms()
    per_kf = n / max(c["keyframes"] - 1, 1)
    gt = np.array([fr[2] for fr in frames])
    from orb_slam2_with_comment_amd.system import ate_rmse
    print(f"{n} frames in {dt * 1e3:.1f} ms ({n / dt:.1f} fps), {c}, ATE {ate_rmse(slam.trajectory_twc(), gt):.4f} m")
    print(f"  local mapping: {slam.local_mapping_counts()}")
    for k, v in ph.items():
        print(f"  {k:24s} {v:8.4f} ms/frame" + (f"  {v * per_kf:8.4f} ms/keyframe" if k.startswith("lm_") else ""))
    slam.Shutdown()


if __name__ == "__main__":
    main()
