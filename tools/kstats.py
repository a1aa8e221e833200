"""Per-kernel totals from a rocprofv3 kernel trace csv: calls, total and average us, share.
Usage: python tools/kstats.py <kernel_trace.csv> [name-filter]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = defaultdict(lambda: [0, 0.0])
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("orbmi::", "").replace("void ", "")
    if flt not in n:
        continue
    agg[n][0] += 1
    agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in agg.values())
for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f"{n[:48]:48s} {c:6d} {t:10.1f} us {t / c:8.2f} us/call {100 * t / tot:5.1f} %")
