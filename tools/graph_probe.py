"""Probe: capture one tracked stereo frame (StereoTracker.track) into a HIP graph through
torch.cuda.graph on the library's stream and compare replay with eager enqueue."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402


class A:
    frames, nfeatures = 4, 2000


S = bench.setup_track(A, 0, 0)
tr = S["tr"]
cam = S["cam"]
rows, cols = cam.height, cam.width
img_bytes = rows * cols
ext = torch.cuda.ExternalStream(tr.stream_handle, device=tr.kps.device)


def track(f):
    tr.track(S["imgs"].data_ptr() + f * 2 * img_bytes, rows, cols, S["tcws"][f], S["lf_views"][f - 1],
             S["lf_pts"][f - 1].data_ptr(), S["mps"][f].data_ptr(), S["n_mp"][f])


for i in range(6):
    track(2 + i % 4)
tr.synchronize()
ref = tr.results()
n = 64
t0 = time.perf_counter()
for i in range(n):
    track(2 + i % 4)
te = (time.perf_counter() - t0) / n * 1e3
tr.synchronize()
tt = (time.perf_counter() - t0) / n * 1e3
print(f"eager: enqueue {te:.3f} ms/frame, total {tt:.3f} ms/frame", flush=True)
graphs = []
for f in range(2, 6):
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=ext):
        track(f)
    graphs.append(g)
print("captured", len(graphs), "graphs", flush=True)
for g in graphs:
    g.replay()
tr.synchronize()
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(n):
    graphs[i % 4].replay()
te = (time.perf_counter() - t0) / n * 1e3
torch.cuda.synchronize()
tr.synchronize()
tt = (time.perf_counter() - t0) / n * 1e3
print(f"graph: enqueue {te:.3f} ms/frame, total {tt:.3f} ms/frame", flush=True)
# same result as eager for the last frame replayed (frame 2 + (n-1) % 4)
track(2 + (n - 1) % 4)
tr.synchronize()
r_e = tr.results()
graphs[(n - 1) % 4].replay()
torch.cuda.synchronize()
r_g = tr.results()
print("parity:", r_e["inliers"] == r_g["inliers"], np.abs(r_e["tcw"] - r_g["tcw"]).max(), flush=True)
