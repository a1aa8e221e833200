"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel mean duration and the idle gaps between
consecutive dispatches on one queue (launch latency evidence for the latency-bound chains).

    python tools/trace_gaps.py <kernel_trace.csv> [name-substring]
"""
import csv
import sys
from collections import defaultdict


def main(path, sub=""):
    rows = [r for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = defaultdict(list)
    gaps = defaultdict(list)
    prev = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
        dur[name].append(e - s)
        if prev is not None and s - prev[1] < 200_000:  # same burst
            gaps[name].append(s - prev[1])
        prev = (s, e, name)
    tot = sum(sum(v) for v in dur.values())
    print(f"{'kernel':48s} {'calls':>6s} {'mean us':>8s} {'gap-before us':>13s}")
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        g = gaps.get(k, [])
        print(f"{k:48s} {len(v):6d} {sum(v) / len(v) / 1e3:8.2f} {(sum(g) / len(g) / 1e3 if g else 0):13.2f}")
    span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"]) if rows else 0
    print(f"busy {tot / 1e3:.1f} us over a span of {span / 1e3:.1f} us")


if __name__ == "__main__":
    main(*sys.argv[1:])
