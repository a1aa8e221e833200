"""Latency of one PoseOptimization launch (k_pose_opt via the device path) for the Track stages'
edge counts, plus the per-wave event timeline of the traced variant (orbmi_debug_pose_trace);
run under rocprofv3 --kernel-trace --stats for per-kernel time."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from orb_slam2_with_comment_amd import synth_map as SM  # noqa: E402
from orb_slam2_with_comment_amd._capi import lib  # noqa: E402
from orb_slam2_with_comment_amd.optimizer import PoseOptimizer  # noqa: E402

SEQS, WAVES = 64, 8

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
    tr = np.zeros(16 + SEQS * WAVES * 8, np.uint64)
    d_fr.copy_(d_fr0)
    torch.cuda.synchronize()
    rc = lib().orbmi_debug_pose_trace(po._h, d_fr.data_ptr(), d_ob.data_ptr(), d_out.data_ptr(), tr.ctypes.data)
    assert rc == 0, rc
    tot, real, nseq = int(tr[0]), int(tr[1]), int(tr[2])
    print(f"  traced: {real / 100.0:.1f} us, {tot} cycles ({tot / (real / 100.0):.0f} MHz), {nseq} passes", flush=True)
    ev = tr[16:].reshape(SEQS, WAVES, 8).astype(np.int64)
    # per trial (seq): pass, chi2 barrier B1, decision; accepted trials add the 28-value
    # reduction (B2), wave 0's lane-parallel trial chain and the candidates barrier B3 (cycles)
    sums = {"trial(wave0)": [], "pass(max wave)": [], "pass(wave0)": [], "B1 wait(wave0)": [],
            "decision(wave0)": [], "reduce+B2(wave0)": [], "  full pass(wave0)": [], "  full pass(max wave)": [],
            "  reduce28+B2(wave0)": [], "chain solve(wave0)": [], "B3 wait(wave1)": []}
    acc_n = 0
    for s in range(1, min(nseq, SEQS) - 1):
        e, nxt = ev[s], ev[s + 1]
        act = [w for w in range(WAVES) if e[w, 0] and e[w, 1]]
        if 0 not in act:
            continue
        if nxt[0, 0]:
            sums["trial(wave0)"].append(nxt[0, 0] - e[0, 0])
        sums["pass(max wave)"].append(max(e[w, 1] - e[w, 0] for w in act))
        sums["pass(wave0)"].append(e[0, 1] - e[0, 0])
        if e[0, 2]:
            sums["B1 wait(wave0)"].append(e[0, 2] - e[0, 1])
        if e[0, 3] and e[0, 2]:
            sums["decision(wave0)"].append(e[0, 3] - e[0, 2])
        if e[0, 4] and e[0, 3]:
            acc_n += 1
            sums["reduce+B2(wave0)"].append(e[0, 4] - e[0, 3])
            if e[0, 7]:
                sums["  full pass(wave0)"].append(e[0, 7] - e[0, 3])
                sums["  reduce28+B2(wave0)"].append(e[0, 4] - e[0, 7])
                sums["  full pass(max wave)"].append(max(e[w, 7] - e[w, 3] for w in act if e[w, 7] and e[w, 3]))
            if e[0, 5]:
                sums["chain solve(wave0)"].append(e[0, 5] - e[0, 4])
            if e[1, 6] and e[1, 3]:
                sums["B3 wait(wave1)"].append(e[1, 6] - e[1, 3])
    print(f"    accepted (or regenerated) trials with a fresh solve: {acc_n}", flush=True)
    for k, v in sums.items():
        if v:
            print(f"    {k:22s} mean {np.mean(v):8.0f} cycles  (n={len(v)})", flush=True)
po.close()
