"""Where the concurrent LocalMapping's accuracy goes when frames come back to back
(VERDICT r04 item 2): the native loop (csrc/slam.cpp, LocalMapping on its own thread) on the
200-frame sequence of tests/test_native_slam_gpu.py, several runs per regime:

  back-to-back              the throughput regime (bench --mode system)
  back-to-back, no interrupt  the same with mbAbortBA never raised (ORBMI_SLAM_NO_INTERRUPT=1)
  paced 3 ms / 6 ms          frames handed over as stereo_kitti.cc:95-107 waits out timestamps

Per run, from the recorded schedule (orbmi_slam_get_schedule) and LocalBA log: keyframes,
keyframes refused (NeedNewKeyFrame true but the queue full), LocalMapping jobs, jobs whose
SearchInNeighbors / LocalBA were skipped because another keyframe was queued (CheckNewKeyFrames,
src/LocalMapping.cc:82-95), LocalBAs run / interrupted mid-run / stopped before starting, ATE.
tests/test_native_slam_gpu.py::test_concurrent_schedule_replays_on_oracle shows that a recorded
run replays on the oracle to the same trajectory, so these counts are the reference logic's.

python tools/concur_breakdown.py [runs]"""
import json
import os
import sys
import time

# as bench.py: 8 hardware queues (the process's streams then map onto queues of their own)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import tempfile  # noqa: E402

import numpy as np  # noqa: E402

from orb_slam2_with_comment_amd.native_slam import NativeStereoSLAM  # noqa: E402
from orb_slam2_with_comment_amd.system import L_BA, L_FUSE_BATCH, L_JOB, ate_rmse  # noqa: E402
from slam_backends import render_sequence, sequence_settings, small_vocabulary  # noqa: E402


def jobs(sched):
    """Per LocalMapping job (keyframe): did SearchInNeighbors / LocalBA run (from the resume
    points the mapping thread logged)."""
    out, cur = [], None
    for t, label, arg in sched.tolist():
        if t != 1:
            continue
        if label == L_JOB:
            if cur is not None:
                out.append(cur)
            cur = {"kf": arg, "sin": False, "ba": False} if arg >= 0 else None
        elif cur is not None and label == L_FUSE_BATCH:
            cur["sin"] = True
        elif cur is not None and label == L_BA:
            cur["ba"] = True
    if cur is not None:
        out.append(cur)
    return out


def run(frames, s, voc, period, no_interrupt):
    if no_interrupt:
        os.environ["ORBMI_SLAM_NO_INTERRUPT"] = "1"
    else:
        os.environ.pop("ORBMI_SLAM_NO_INTERRUPT", None)
    slam = NativeStereoSLAM(s, device=0, vocabulary=voc, async_local_mapping=True, record=True)
    t0 = time.perf_counter()
    for f, (L, R, _) in enumerate(frames):
        nxt = frames[f + 1][:2] if f + 1 < len(frames) else None
        slam.TrackStereo(L, R, 0.1 * f, next_pair=nxt)
        wait = t0 + (f + 1) * period - time.perf_counter()
        if wait > 0:
            time.sleep(wait)
    el = time.perf_counter() - t0
    slam.WaitLocalMapping()
    gt = np.array([fr[2] for fr in frames])
    ate = ate_rmse(slam.trajectory_twc(), gt)
    st, sched, ba, c = slam.stats, slam.schedule(), slam.local_ba_log(), slam.counts()
    lmc = slam.local_mapping_counts()
    ph = slam.phase_ms()
    per_kf = len(frames) / max(c["keyframes"] - 1, 1)
    slam.Shutdown()
    refused = 0
    for a, b in zip(st, st[1:]):
        if b.get("need_kf") and b.get("keyframes") == a.get("keyframes"):
            refused += 1
    jb = jobs(sched)
    return {"ate_m": round(ate, 4), "frames_per_s": round(len(frames) / el, 1), "keyframes": c["keyframes"],
            "refused": refused, "jobs": len(jb), "sin_skipped": sum(not j["sin"] for j in jb),
            "ba_skipped": sum(not j["ba"] for j in jb), "local_ba": int(len(ba)),
            "ba_interrupted": int((ba[:, 1] > 0).sum()) if len(ba) else 0,
            "ba_aborted_before_start": int((ba[:, 1] == 0).sum()) if len(ba) else 0,
            "lm_ms_per_keyframe": round(ph["lm_total"] * per_kf, 3), "lm_lock_wait_ms_per_keyframe":
            round(ph["lm_lock_wait"] * per_kf, 3), "native_counts": lmc}


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    frames = render_sequence(200)
    s = sequence_settings(tempfile.mkdtemp())
    voc = small_vocabulary()
    regimes = [("back-to-back", 0.0, False), ("back-to-back, no interrupt", 0.0, True), ("paced 3 ms", 0.003, False),
               ("paced 6 ms", 0.006, False)]
    out = {}
    for name, period, noint in regimes:
        rs = [run(frames, s, voc, period, noint) for _ in range(runs)]
        out[name] = rs
        keys = list(rs[0])
        print(f"{name}:", flush=True)
        for k in keys:
            print(f"  {k:28s} " + "  ".join(f"{str(r[k]):>8}" for r in rs), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
