#!/usr/bin/env python3
"""Per-kernel durations and the idle gaps between consecutive kernels from a
rocprofv3 --kernel-trace CSV (…kernel_trace.csv).

usage: python tools/kgaps.py DIR [name-substring ...]

Prints, for each kernel name, the mean duration, and for each ordered pair of
consecutive kernels (on the same queue) the mean gap end(prev) -> start(next),
so the time per bench step that no kernel covers is visible.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(n):
    return n.split("(")[0].replace("void ", "").replace("na::", "").strip()


def main():
    d = sys.argv[1]
    subs = sys.argv[2:]
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                             r.get("Queue_Id", "0")))
    rows.sort()
    if subs:
        rows = [r for r in rows if any(s in r[2] for s in subs)]
    dur = defaultdict(list)
    gap = defaultdict(list)
    for i, (s, e, n, q) in enumerate(rows):
        dur[n].append((e - s) / 1e3)
        if i:
            ps, pe, pn, pq = rows[i - 1]
            g = (s - pe) / 1e3
            if 0 <= g < 1000:  # skip host-side pauses between phases
                gap[(pn, n)].append(g)
    for n, v in dur.items():
        v = sorted(v)
        print(f"{n:48s} n={len(v):4d} mean {sum(v)/len(v):8.2f} us  p50 {v[len(v)//2]:8.2f}")
    for (a, b), v in gap.items():
        if len(v) >= 5:
            v = sorted(v)
            print(f"gap {a[:30]:30s} -> {b[:30]:30s} n={len(v):4d} mean {sum(v)/len(v):6.2f} us  p50 {v[len(v)//2]:6.2f}")


if __name__ == "__main__":
    main()
