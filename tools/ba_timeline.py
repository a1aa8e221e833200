"""Timeline of one LocalBundleAdjustment call from a rocprofv3 kernel trace (csv): per-kernel
durations and the gaps between them.  Usage: python tools/ba_timeline.py <kernel_trace.csv> [call]"""
import csv
import sys
from collections import defaultdict

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_ba_" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_ba_setup" in r["Kernel_Name"]]
call = int(sys.argv[2]) if len(sys.argv) > 2 else len(starts) // 2
i0 = starts[call]
i1 = starts[call + 1] if call + 1 < len(starts) else len(rows)
t0 = int(rows[i0]["Start_Timestamp"])
prev = t0
tot = defaultdict(float)
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("orbmi::", "")
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:6.1f} gap {(s - prev) / 1e3:5.1f}  {name}")
    tot[name] += (e - s) / 1e3
    tot["(gaps)"] += (s - prev) / 1e3
    prev = e
print(f"call span {(prev - t0) / 1e3:.1f} us")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"  {k:24s} {v:8.1f} us")
