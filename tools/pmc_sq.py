"""Per-kernel sums of rocprofv3 PMC counters (counter_collection CSVs under DIR, any pass).

    python tools/pmc_sq.py DIR [kernel-filter]

Prints, per kernel: launches and the per-launch mean of every counter collected.  SQ cycle
counters (SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_*, SQ_BUSY_CYCLES) are quad-cycles on gfx950
(MI355X_MICROARCH.md, per-instruction constants)."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
vals = defaultdict(lambda: defaultdict(float))
disp = defaultdict(lambda: defaultdict(set))
for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "")
        m = re.search(r"(k_\w+)", name)
        k = m.group(1) if m else name[:40]
        if flt and flt not in k:
            continue
        c = row["Counter_Name"]
        vals[k][c] += float(row["Counter_Value"])
        disp[k][c].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
for k in sorted(vals):
    print(k)
    for c in sorted(vals[k]):
        n = max(len(disp[k][c]), 1)
        print(f"   {c:28s} {vals[k][c] / n:16.1f} per launch  ({n} launches)")
