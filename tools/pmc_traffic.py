"""Summarise rocprofv3 PMC runs into per-kernel HBM bytes per launch.

    python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json [CONFIG_JSON]

CONFIG_JSON (`python bench.py --print-traffic-config <the run's args>`) is stored as "config":
bench.py reports a summary as roofline.traffic only for a run of the same workload.

FETCH_DIR / WRITE_DIR hold the counter_collection CSVs of two separate passes
(`rocprofv3 --pmc FETCH_SIZE --kernel-trace ...`, `--pmc WRITE_SIZE ...`).  Per
MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the
bytes read, so bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024.  Calibrated on this pool for coalesced
4-, 8- and 16-byte loads and stores per lane (tools/ubench/fetch_calib.hip,
profiles/r04/fetch_calibration.txt: FETCH_SIZE x2.000 and WRITE_SIZE x1.000 at every width).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

STAGE_OF = [("k_pyramid", "pyr_level0"), ("k_pyr_level0", "pyr_level0"), ("k_pyr_resize", "pyr_resize"), ("k_fast", "fast"),
            ("k_octree", "octree"), ("k_describe", "describe"), ("k_stereo_rows", "stereo_rows"),
            ("k_stereo_match", "stereo_match"), ("k_stereo_filter", "stereo_filter")]


def stage(name):
    """Bench stage name for the extractor kernels, the kernel's own name (k_...) otherwise."""
    import re
    for k, s in STAGE_OF:
        if k in name:
            return s
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else None


def read(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            s = stage(row.get("Kernel_Name", ""))
            if s:
                vals[s].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items() if v}


def main(fetch_dir, write_dir, out, config=None):
    fetch = read(fetch_dir, "FETCH_SIZE")
    write = read(write_dir, "WRITE_SIZE")
    per = {}
    raw = {}
    for s in sorted(set(fetch) | set(write)):
        f = fetch.get(s, 0.0)
        w = write.get(s, 0.0)
        per[s] = round((2 * f + w) * 1024)
        raw[s] = {"FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w}
    json.dump({"per_launch_bytes": per, "raw_per_launch": raw, "config": json.loads(config) if config else None,
               "note": "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE half count, calibrated for 4/8/16-B loads: profiles/r04/fetch_calibration.txt)"},
              open(out, "w"), indent=1)
    print(json.dumps(per))


if __name__ == "__main__":
    main(*sys.argv[1:5])
