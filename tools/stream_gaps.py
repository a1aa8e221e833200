"""Kernel durations and inter-kernel gaps on the tracking stream (the stream running k_pose_opt)
of a rocprofv3 --kernel-trace directory, over the last 1100 kernels (the timed region):
python tools/stream_gaps.py DIR"""
import collections
import csv
import glob
import statistics
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
by = collections.defaultdict(list)
for r in rows:
    by[(r["Queue_Id"], r["Stream_Id"])].append(r)
key = next(k for k, v in by.items() if any("k_pose_opt" in x["Kernel_Name"] for x in v))
v = sorted(by[key], key=lambda r: r["s"])[-1100:]
dur = collections.defaultdict(list)
for r in v:
    dur[r["Kernel_Name"][:26]].append((r["e"] - r["s"]) / 1e3)
print("kernel durations (us, median):", {k: (len(x), round(statistics.median(x), 2)) for k, x in dur.items()})
gaps = collections.defaultdict(list)
for a, b in zip(v, v[1:]):
    g = (b["s"] - a["e"]) / 1e3
    if g < 40:
        gaps[(a["Kernel_Name"][:16], b["Kernel_Name"][:16])].append(g)
print("gaps (us, median):", {f"{a}->{b}": (len(g), round(statistics.median(g), 2)) for (a, b), g in gaps.items() if len(g) > 20})
