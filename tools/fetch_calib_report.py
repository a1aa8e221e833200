"""Counter-to-byte factors per access width from tools/ubench/fetch_calib under rocprofv3
(FETCH_SIZE and WRITE_SIZE passes): bytes / (counter KiB * 1024) per kernel, second repetition."""
import csv
import glob
import os
import sys
from collections import defaultdict

BYTES = 512 << 20


def read(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") == counter:
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def main(fdir, wdir):
    for d, c, pre in ((fdir, "FETCH_SIZE", "k_read"), (wdir, "WRITE_SIZE", "k_write")):
        for k, v in sorted(read(d, c).items()):
            if pre not in k:
                continue
            kib = v[-1]
            print(f"{c:10s} {k[:40]:40s} {kib:14.1f} KiB  bytes / (counter * 1024) = {BYTES / (kib * 1024):.3f}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
