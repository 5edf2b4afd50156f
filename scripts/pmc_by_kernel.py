#!/usr/bin/env python3
"""pmc_by_kernel.py — mean of each rocprofv3 PMC counter per dispatch, per
kernel name, over one or more pmc_counter_collection.csv files (separate
--pmc passes). FETCH_SIZE is reported doubled as `fetch_bytes` (gfx950:
FETCH_SIZE counts half of a wide streaming read, MI355X_MICROARCH.md §HBM) and
WRITE_SIZE as `write_bytes` (KiB -> bytes).
usage: pmc_by_kernel.py <csv> [<csv> ...]   (prints JSON)
"""
import collections
import csv
import json
import sys


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in sys.argv[1:]:
        with open(path) as f:
            for r in csv.DictReader(f):
                acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        row = {c: sum(v) / len(v) for c, v in cs.items()}
        row["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in row:
            row["fetch_bytes"] = 2 * row["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in row:
            row["write_bytes"] = row["WRITE_SIZE"] * 1024
        if "TCC_HIT_sum" in row and "TCC_MISS_sum" in row:
            row["l2_hit_rate"] = row["TCC_HIT_sum"] / max(1.0, row["TCC_HIT_sum"] + row["TCC_MISS_sum"])
        out[k] = row
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
