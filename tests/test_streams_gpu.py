"""Config 4 executed: two ranks, each tracking its own KITTI-shaped stereo
stream with the pipelined StereoTracker, exchange every frame's left keypoints + descriptors with
pipeline.StreamExchange and match them against the other stream's (build-defined cross-stream
matching; the partition rationale is src/Tracking.cc:997-1063, every stream's frame t depends on
its own map at t-1, so streams are replicas and the exchange is the only collective).

The 1-GPU box cannot hold two RCCL ranks on one device, so the ranks run the exchange over a gloo
group with CUDA tensors, both on cuda:0; the code path (StreamExchange on its own stream X, the
slot holds of the double-buffered tracker, the match kernel) is the one the RCCL run executes.

Checked per step, against independent references:
  * every gathered segment s equals the oracle's extraction of stream s's left image of THAT
    step's frame (keypoints and descriptors bit-exact, count exact).  A slot overwritten by the
    extraction two frames later before the gather read it would show the wrong frame's features
    (the round-1 race on hold_slot);
  * the rank's cross-stream matches equal oracle.match_descriptors_segments on the gathered data.
And bench.py --gpus 2 --dist-backend gloo prints a config-4 line with cross-stream matches."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEPS = 10
FRAMES = 4  # distinct resident frames per stream (bench.setup_track); steps cycle through them


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        import argparse

        import torch
        import torch.distributed as dist
        sys.path.insert(0, ROOT)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import bench
        from orb_slam2_with_comment_amd.pipeline import StreamExchange
        S = bench.setup_track(argparse.Namespace(frames=FRAMES, nfeatures=2000), rank, 0)
        tr = S["tr"]
        cam = S["cam"]
        rows, cols = cam.height, cam.width
        xch = StreamExchange(tr, dist, 0)
        hist = []
        for i in range(STEPS):
            f = 2 + i % FRAMES
            tr.track(S["imgs"].data_ptr() + f * 2 * rows * cols, rows, cols, S["tcws"][f], S["lf_views"][f - 1],
                     S["lf_pts"][f - 1].data_ptr(), S["mps"][f].data_ptr(), S["n_mp"][f])
            g_desc, g_kps, g_cnt = xch.exchange()
            with torch.cuda.stream(xch.X):  # snapshots ordered after the gather and the match on X
                hist.append((f, g_desc.clone(), g_kps.clone(), g_cnt.clone(), xch.xmatch.clone()))
        tr.synchronize()
        xch.synchronize()
        torch.cuda.synchronize()
        out = [(f, d.cpu().numpy(), k.cpu().numpy(), c.cpu().numpy().reshape(-1), m.cpu().numpy())
               for f, d, k, c, m in hist]
        q.put((rank, out, None))
        dist.barrier()
        xch.close()
        tr.close()
        dist.destroy_process_group()
    except Exception as e:  # surfaced in the parent
        import traceback
        q.put((rank, None, traceback.format_exc() + repr(e)))


def test_stream_exchange_two_ranks(oracle):
    import torch.multiprocessing as mp
    from orb_slam2_with_comment_amd import synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, out, err = q.get(timeout=300)
        assert err is None, err
        res[r] = out
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    p_or = oracle.params(2000)
    ref = {}  # (stream, frame) -> oracle keypoints (n x 7 int32 view), descriptors
    for s in range(2):
        for f in range(2, 2 + FRAMES):
            L, _, _ = synth.stereo_pair(synth.KITTI, f, seed_base=1000 * (s + 1))
            k, d = oracle.extract(p_or, L)
            ref[s, f] = (np.ascontiguousarray(k).view(np.int32).reshape(len(k), 7), d)
    total_x = 0
    for rank in range(2):
        assert len(res[rank]) == STEPS
        for i, (f, g_desc, g_kps, g_cnt, xm) in enumerate(res[rank]):
            assert f == 2 + i % FRAMES
            for s in range(2):
                rk, rd = ref[s, f]
                n = len(rk)
                assert int(g_cnt[s]) == n, (rank, i, s, int(g_cnt[s]), n)
                np.testing.assert_array_equal(g_kps[s, :n], rk, err_msg=f"rank {rank} step {i} segment {s}")
                np.testing.assert_array_equal(g_desc[s, :n], rd, err_msg=f"rank {rank} step {i} segment {s}")
            n_own = int(g_cnt[rank])
            want = oracle.match_descriptors_segments(g_desc[rank, :n_own], g_desc, g_cnt, rank, 50, 0.6)
            np.testing.assert_array_equal(xm[:n_own], want, err_msg=f"rank {rank} step {i} cross matches")
            # matches point into the OTHER stream's segment
            hit = xm[:n_own] >= 0
            cap = g_desc.shape[1]
            assert (xm[:n_own][hit] // cap != rank).all()
            total_x += int(hit.sum())
    # the streams see the same world (different sensor noise): most features re-observed
    assert total_x > 2 * STEPS * 500, total_x


def test_bench_config4_gloo_two_ranks(tmp_path):
    """bench.py's N > 1 path end to end at world size 2 (gloo rehearsal on one device)."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--mode", "track", "--gpus", "2", "--dist-backend", "gloo",
           "--steps", "12", "--warmup", "4", "--frames", "4", "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    log_dir = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(log_dir):
        with open(os.path.join(log_dir, "bench_config4_gloo.json"), "w") as fh:
            fh.write(lines[0] + "\n")
    assert out["n_gpus"] == 2 and out["scaling"] == "weak"
    assert out["cross_stream_matches_last_frame"] > 0
    assert out["matches_per_frame"]["tracking_ok"]
    assert "config 4" in out["config"]["workload"]
