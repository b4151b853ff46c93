#!/usr/bin/env python3
"""The C5 step's kernel timeline from a rocprofv3 --kernel-trace CSV of
`bench.py --config c5` (two streams): for the last N steps, each kernel's
start/end relative to the step's first kernel, the step span, the kernel
sum, and the overlap (sum / span).  VERDICT r4 item 1 asks for the halves
to overlap (step <= 0.8 x the kernel sum).

usage: python tools/c5_timeline.py DIR [steps]
"""
import csv
import glob
import os
import sys


def short(n):
    return n.split("(")[0].replace("void ", "").replace("na::", "").strip()


def main():
    d = sys.argv[1]
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                n = short(r["Kernel_Name"])
                if any(x in n for x in ("gcm_ragged", "seg_", "chachapoly_")):
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n))
    rows.sort()
    # a step = the AES seal launch and everything until the next one
    starts = [i for i, r in enumerate(rows) if r[2].startswith("gcm_ragged_staged<false")]
    steps = []
    for a, b in zip(starts, starts[1:] + [len(rows)]):
        steps.append(rows[a:b])
    # whole steps only (bench's per-kernel timing pass afterwards runs each
    # kernel alone): both ciphers' seal and open
    steps = [st for st in steps if len({r[2] for r in st if not r[2].startswith("seg_plan")}) >= 4]
    spans, sums = [], []
    for st in steps[-nsteps:]:
        t0 = min(r[0] for r in st)
        t1 = max(r[1] for r in st)
        ksum = sum(r[1] - r[0] for r in st if not r[2].startswith("seg_plan"))
        spans.append((t1 - t0) / 1e3)
        sums.append(ksum / 1e3)
        print(f"step: span {(t1 - t0) / 1e3:.1f} us, kernel sum {ksum / 1e3:.1f} us, span/sum {(t1 - t0) / ksum:.3f}")
        for s, e, n in st:
            print(f"   {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f}  {(e - s) / 1e3:7.1f}  {n}")
    if spans:
        print(f"mean span {sum(spans) / len(spans):.1f} us, mean kernel sum {sum(sums) / len(sums):.1f} us, "
              f"ratio {sum(spans) / sum(sums):.3f}")


if __name__ == "__main__":
    main()
