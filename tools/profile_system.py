"""cProfile of the StereoSLAM host loop on the GPU backend (host-side hot spots of --mode system).
Usage: python tools/profile_system.py [frames]"""
import cProfile
import os
import pstats
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (HIP runtime before liborbmi.so)

from orb_slam2_with_comment_amd import synth  # noqa: E402
from orb_slam2_with_comment_amd.settings import load_settings, write_settings  # noqa: E402
from orb_slam2_with_comment_amd.system import StereoSLAM  # noqa: E402
from orb_slam2_with_comment_amd.vocabulary import Vocabulary  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
frames = [synth.stereo_pair(synth.KITTI, f) for f in range(n)]
path = os.path.join(tempfile.mkdtemp(), "k.yaml")
write_settings(path, synth.KITTI)
slam = StereoSLAM(load_settings(path), device=0, vocabulary=Vocabulary.synthetic(k=10, L=5, seed=3))
for f in range(4):
    slam.TrackStereo(frames[f][0], frames[f][1], 0.1 * f)
pr = cProfile.Profile()
t = time.perf_counter()
pr.enable()
for f in range(4, n):
    slam.TrackStereo(frames[f][0], frames[f][1], 0.1 * f)
pr.disable()
print(f"{(time.perf_counter() - t) / (n - 4) * 1e3:.2f} ms/frame")
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
