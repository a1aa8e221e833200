"""Hunt for a concurrent-schedule replay mismatch (tests/test_native_slam_gpu.py::
test_concurrent_schedule_replays_on_oracle) and localise it.

    python tools/replay_hunt.py [runs] [period[,period...]] [both]

Records up to `runs` concurrent native runs (200 frames, frames `period` s apart, the periods
taken in turn when several are given) and replays
each on the CPU oracle (system.StereoSLAM.replay_schedule with the per-keyframe state record).
At the first mismatch it replays the same record with the GPU operators behind the same Python
host logic (GpuBackend: the GPU searches, the host triangulation): if that replay agrees with the
native record where the oracle's did not, the oracle and the GPU operators disagree on that input;
if it stops at the same place with the oracle's values, the native run's device call (or its
inputs) differs.  The record goes to gpurun_out/replay_hunt.npz.  `both`: every run is also replayed with the GPU
operators (which must then be exact too), to exercise that path without waiting for a mismatch."""
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

from slam_backends import OracleBackend, render_sequence, sequence_settings, small_vocabulary  # noqa: E402
from orb_slam2_with_comment_amd.native_slam import NativeStereoSLAM  # noqa: E402
from orb_slam2_with_comment_amd.system import ScheduleMismatch, StereoSLAM  # noqa: E402


def drive(slam, frames, period):
    t0 = time.perf_counter()
    for f, (L, R, _) in enumerate(frames):
        nxt = frames[f + 1][:2] if f + 1 < len(frames) else None
        slam.TrackStereo(L, R, 0.1 * f, next_pair=nxt)
        wait = t0 + (f + 1) * period - time.perf_counter()
        if wait > 0:
            time.sleep(wait)


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    periods = [float(p) for p in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0.003]
    both = len(sys.argv) > 3 and sys.argv[3] == "both"
    frames = render_sequence(200)
    voc = small_vocabulary()
    tmp = tempfile.mkdtemp()
    s = sequence_settings(__import__("pathlib").Path(tmp))
    replay_frames = [(L, R, 0.1 * f) for f, (L, R, _) in enumerate(frames)]
    for run in range(runs):
        period = periods[run % len(periods)]
        slam = NativeStereoSLAM(s, device=0, vocabulary=voc, async_local_mapping=True, record=True)
        drive(slam, frames, period)
        slam.WaitLocalMapping()
        rec = {"schedule": slam.schedule(), "ba_log": slam.local_ba_log(), "kf_state": slam.keyframe_state_log()}
        counts = slam.counts()
        slam.Shutdown()
        ref = StereoSLAM(s, backend=OracleBackend(s, voc))
        try:
            ref.replay_schedule(replay_frames, rec["schedule"], rec["ba_log"], rec["kf_state"])
            print(f"run {run} (period {period}): replay exact ({len(rec['schedule'])} events, {counts})", flush=True)
            if both:
                gpu = StereoSLAM(s, device=0, vocabulary=voc)
                try:
                    gpu.replay_schedule(replay_frames, rec["schedule"], rec["ba_log"], rec["kf_state"])
                    d = float(np.abs(gpu.trajectory_twc() - ref.trajectory_twc()).max())
                    print(f"  GPU-operator replay: exact; its trajectory vs the oracle replay's: max |d| {d:.3g}",
                          flush=True)
                except ScheduleMismatch as e:
                    print(f"  GPU-operator replay mismatch: {e}", flush=True)
                    return 1
                finally:
                    gpu.backend.close()
            continue
        except ScheduleMismatch as e:
            print(f"run {run} (period {period}): ORACLE replay mismatch: {e}", flush=True)
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        np.savez(os.path.join(ROOT, "gpurun_out", "replay_hunt.npz"), schedule=rec["schedule"], ba_log=rec["ba_log"],
                 kf_state=rec["kf_state"], period=period)
        gpu = StereoSLAM(s, device=0, vocabulary=voc)
        try:
            gpu.replay_schedule(replay_frames, rec["schedule"], rec["ba_log"], rec["kf_state"])
            print("  GPU-operator replay: exact -> the oracle and the GPU operators disagree on that input", flush=True)
        except ScheduleMismatch as e:
            print(f"  GPU-operator replay mismatch: {e}", flush=True)
        return 1
    print("no mismatch in", runs, "runs")
    return 0


if __name__ == "__main__":
    sys.exit(main())
