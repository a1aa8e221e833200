#!/usr/bin/env python
"""bench.py — MI355X ORB front-end throughput (BASELINE.json metric, config 2 workload).

One step = one KITTI-shaped 1241x376 stereo frame through the GPU hot path:
ORBextractor on the left and right images (2000 features, 8 levels; one batched launch
sequence) + Frame::ComputeStereoMatches.  Frames are synthetic (ray-cast KITTI-shaped
sequence, orb_slam2_with_comment_amd/synth.py) and resident in HBM before timing.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, weak scaling:
        every rank runs its own stereo stream; no data-path collective)

Prints ONE JSON line on rank 0 (contract in the task statement / DESIGN.md §Measurement).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (loaded before liborbmi.so: one HIP runtime in the process)

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--frames", type=int, default=8, help="distinct stereo frames resident per rank")
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--cpu-sample-s", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="per-stage PMC HBM bytes (written by tools/pmc_traffic.py)")
    return ap.parse_args()


def level_geometry(orb_mod, rows, cols, nlevels=8, sf=1.2):
    """Pyramid sizes exactly as ComputePyramid (cvRound((float)cols * invScale))."""
    s = np.float32(1.0)
    W, H = [], []
    for _ in range(nlevels):
        inv = np.float32(1.0) / s
        W.append(int(np.rint(np.float32(cols) * inv)))
        H.append(int(np.rint(np.float32(rows) * inv)))
        s = np.float32(np.float64(s) * np.float64(np.float32(sf)))
    return W, H


def main():
    a = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from orb_slam2_with_comment_amd import _capi, synth
    from orb_slam2_with_comment_amd.orb import ORBextractor

    lib = _capi.lib()
    cam = synth.KITTI
    rows, cols = cam.height, cam.width
    # every rank owns one stereo stream (weak scaling); frames resident in HBM
    frames = [synth.stereo_pair(cam, f, seed_base=1000 * (rank + 1))[:2] for f in range(a.frames)]
    host = np.stack([np.stack(p) for p in frames])  # F x 2 x H x W
    d_img = torch.from_numpy(host).cuda()
    ex = ORBextractor(a.nfeatures, 1.2, 8, 20, 7, device=local)
    cap = a.nfeatures + 64
    d_kps = torch.zeros((2, cap, 7), dtype=torch.int32, device="cuda")
    d_desc = torch.zeros((2, cap, 32), dtype=torch.uint8, device="cuda")
    d_cnt = torch.zeros(2, dtype=torch.int32, device="cuda")
    d_u = torch.zeros((2, cap), dtype=torch.float32, device="cuda")
    d_d = torch.zeros((2, cap), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    img_bytes = rows * cols
    vp = C.c_void_p

    def step(i):
        f = i % a.frames
        _capi.check("extract", lib.orbmi_extract_batch_device(
            ex.handle, vp(d_img.data_ptr() + f * 2 * img_bytes), 2, rows, cols, cols, img_bytes,
            vp(d_kps.data_ptr()), vp(d_desc.data_ptr()), vp(d_cnt.data_ptr()), cap))
        _capi.check("stereo", lib.orbmi_compute_stereo_matches_batch_device(
            ex.handle, cam.bf, cam.fx, vp(d_u.data_ptr()), vp(d_d.data_ptr())))

    def sync():
        _capi.check("sync", lib.orbmi_extractor_synchronize(ex.handle))
        torch.cuda.synchronize()

    for i in range(a.warmup):
        step(i)
    sync()

    # ---- per-stage profile pass (untimed): all stages, one cycle over the frame set
    NS = _capi.NUM_STAGES
    ms = np.zeros(NS)
    nl = np.zeros(NS, np.int64)
    lib.orbmi_set_profiling(ex.handle, 0xFF)
    kp_total = 0
    n_prof = max(a.frames, 16)
    for i in range(n_prof):
        step(i)
        sync()
        kp_total += int(d_cnt.sum().item())
    _capi.check("prof", lib.orbmi_read_profile(ex.handle, _capi.ptr(ms), _capi.ptr(nl)))
    lib.orbmi_set_profiling(ex.handle, 0)
    stage_ms_per_step = {(_capi.STAGES[s] if s < len(_capi.STAGES) else str(s)): round(ms[s] / n_prof, 5)
                         for s in range(NS) if nl[s]}
    dom = int(np.argmax(ms))
    kp_per_frame = kp_total / n_prof

    # algorithmic bytes per launch of each stage
    W, H = level_geometry(None, rows, cols)
    P = sum(w * h for w, h in zip(W, H))
    padded = [(w + 38) * (h + 38) for w, h in zip(W, H)]
    n_img = 2
    cand = 0
    for f in range(a.frames):  # FAST candidates (reads the debug view of the last run per frame)
        step(f)
        sync()
        for item in range(2):
            for l in range(8):
                buf = np.zeros((1 << 16, 3), np.int32)
                n = C.c_int()
                lib.orbmi_debug_fast_candidates(ex.handle, item, l, _capi.ptr(buf), 1 << 16, C.byref(n))
                cand += n.value
    cand_per_img = cand / (2 * a.frames)
    kp_per_img = kp_per_frame / 2
    alg = {
        0: n_img * (W[0] * H[0] + padded[0]),                                   # pyr level 0
        1: n_img * sum(W[l - 1] * H[l - 1] + padded[l] for l in range(1, 8)) / 7,  # per resize launch
        2: n_img * (P + 4 * cand_per_img),                                      # FAST: pixels + candidates
        3: n_img * (4 * cand_per_img + 8 * kp_per_img),                         # octree: candidates in, keys out
        4: n_img * kp_per_img * (43 * 43 + 60),                                 # describe: window + kp+desc
    }
    dom_name = _capi.STAGES[dom]

    # ---- timed region: K steps, events bracket the dominant kernel's launches
    lib.orbmi_set_profiling(ex.handle, 1 << dom)
    ms[:] = 0
    nl[:] = 0
    _capi.check("prof", lib.orbmi_read_profile(ex.handle, _capi.ptr(ms), _capi.ptr(nl)))
    ms[:] = 0
    nl[:] = 0
    sync()
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(i)
    sync()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    dt = t1 - t0
    _capi.check("prof", lib.orbmi_read_profile(ex.handle, _capi.ptr(ms), _capi.ptr(nl)))
    lib.orbmi_set_profiling(ex.handle, 0)
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    frames_total = a.steps * world
    value = frames_total / dt
    avg_launch_s = ms[dom] / max(nl[dom], 1) / 1e3
    achieved = alg.get(dom, 0.0) / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    traffic = None
    if os.path.exists(a.traffic):
        try:
            tj = json.load(open(a.traffic))
            traffic = tj.get("per_launch_bytes", {}).get(dom_name)
        except Exception:
            traffic = None

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    cpu = None
    if not a.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(frames, cam, a)

    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: ray-cast KITTI-shaped 1241x376 stereo sequence, resident in HBM",
        "config": {
            "workload": "config2: per step one stereo frame -> ORBextractor(left,right) [2000 feat, 1.2, 8 levels, "
                        "FAST 20/7] + Frame::ComputeStereoMatches; batch=1 frame",
            "frames_resident": a.frames,
            "parallelism": f"replica-per-gpu x{world} (independent stereo streams)",
        },
        "kpts_desc_per_s": round(value * kp_per_frame, 1),
        "keypoints_per_frame": round(kp_per_frame, 1),
        "stage_ms_per_step": stage_ms_per_step,
        "roofline": {
            "kernel": dom_name,
            "bound": "hbm",
            "achieved": round(achieved, 3),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 6),
            "traffic": traffic,
            "alg_bytes_per_launch": round(alg.get(dom, 0.0)),
            "avg_launch_us": round(avg_launch_s * 1e6, 3),
            "launches": int(nl[dom]),
        },
        "pipeline_roofline": {
            "alg_bytes_per_image": 7 * P + 60 * kp_per_img,  # B = 7P + 60N
            "extract_ms_per_step": round(sum(ms_ for k, ms_ in stage_ms_per_step.items()
                                             if k in ("pyr_level0", "pyr_resize", "fast", "octree", "describe")), 5),
        },
        "cpu_baseline": cpu,
        "host": {"cpu": platform.processor() or platform.machine(), "nproc": os.cpu_count(),
                 "hip": torch.version.hip},
    }
    pr = out["pipeline_roofline"]
    if pr["extract_ms_per_step"] > 0:
        gbs = 2 * pr["alg_bytes_per_image"] / (pr["extract_ms_per_step"] / 1e3) / 1e9
        pr["achieved_GBs"] = round(gbs, 3)
        pr["frac"] = round(gbs / HBM_PEAK_GBS, 6)
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def cpu_baseline(frames, cam, a):
    """Oracle (C++ restatement of the reference path) on host cores: L/R extraction on two
    threads (src/Frame.cc:78-81) + ComputeStereoMatches, over a bounded frame sample."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle_ctypes as O
    p = O.params(a.nfeatures)
    pool = ThreadPoolExecutor(2)
    n = 0
    t0 = time.perf_counter()
    while True:
        L, R = frames[n % len(frames)]
        fl = pool.submit(O.extract, p, L)
        fr = pool.submit(O.extract, p, R)
        (kl, dl), (kr, dr) = fl.result(), fr.result()
        O.stereo(p, L, R, cam.bf, cam.fx, kl, dl, kr, dr)
        n += 1
        el = time.perf_counter() - t0
        if (el >= a.cpu_sample_s and n >= 3) or n >= 10000:
            break
    pool.shutdown()
    return {"value": round(n / el, 4), "unit": "frames/s", "cores": 2, "kind": "port",
            "sample": f"{n} KITTI-shaped stereo frames (same synthetic frames), oracle extract L||R "
                      f"(2 threads) + stereo, {el:.1f} s"}


if __name__ == "__main__":
    main()
