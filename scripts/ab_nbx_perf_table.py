#!/usr/bin/env python3
"""ab_nbx_perf_table.py DIR — tabulate nbx_perf_<lib>_d<devs>_rep<k>.txt files
(scripts/steps/r6g.sh, r6h.sh): per rank count and size, the best of the reps'
per-call µs for each library variant, and the wrong-element count."""
import collections
import glob
import os
import re
import sys


def main(d):
    data = collections.defaultdict(list)
    libs = []
    for f in sorted(glob.glob(os.path.join(d, "nbx_perf_*.txt"))):
        m = re.match(r"nbx_perf_(\w+?)_d(\d+)_rep(\d)\.txt", os.path.basename(f))
        if not m:
            continue
        lib, dv, _ = m.groups()
        if lib not in libs:
            libs.append(lib)
        for line in open(f):
            p = line.split()
            if len(p) >= 9 and p[0].isdigit():
                data[(lib, len(dv))].append((int(p[0]), float(p[4]), int(p[7])))
    for n in sorted({k[1] for k in data}):
        print(f"ranks {n}: bytes  " + "  ".join(libs) + "  (us per call, best of reps)  wrong")
        sizes = sorted({s for lib in libs for s, _, _ in data[(lib, n)]})
        for s in sizes:
            cells, wrong = [], 0
            for lib in libs:
                ts = [t for (sz, t, w) in data[(lib, n)] if sz == s]
                wrong += sum(w for (sz, t, w) in data[(lib, n)] if sz == s)
                cells.append(f"{min(ts):9.2f}" if ts else "        -")
            print(f"{s:>11} " + " ".join(cells) + f"  {wrong}")


if __name__ == "__main__":
    main(sys.argv[1])
