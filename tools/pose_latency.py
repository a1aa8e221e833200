"""Latency of one PoseOptimization launch (k_pose_gather + k_pose_opt via the device path) for
the Track stages' edge counts; run under rocprofv3 --kernel-trace --stats for per-kernel time."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from orb_slam2_with_comment_amd import synth_map as SM  # noqa: E402
from orb_slam2_with_comment_amd.optimizer import PoseOptimizer  # noqa: E402

po = PoseOptimizer(0)
for n in (420, 680):
    fr, ob, _ = SM.pose_problem(seed=3, n_obs=n, stereo_frac=0.75, outlier_frac=0.08)
    d_fr0 = torch.from_numpy(fr.view(np.uint8).copy()).cuda()
    d_fr = d_fr0.clone()
    d_ob = torch.from_numpy(ob.view(np.uint8).copy()).cuda()
    d_out = torch.zeros(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    reps = 200
    t0 = time.perf_counter()
    for _ in range(reps):
        d_fr.copy_(d_fr0)
        torch.cuda.synchronize()
        po.run_device(d_fr.data_ptr(), 1, d_ob.data_ptr(), n, d_out.data_ptr())
        po.synchronize()
    dt = (time.perf_counter() - t0) / reps
    res = d_fr.cpu().numpy().view(fr.dtype)
    print(f"n_obs={n}: {dt * 1e6:.1f} us per synchronous launch, iterations={res[0]['iterations']}, "
          f"inliers={res[0]['inliers']}", flush=True)
po.close()
