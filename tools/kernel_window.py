#!/usr/bin/env python3
"""Per-kernel statistics of the TIMED dispatches of a profiled bench.py run.

rocprofv3 --stats averages every dispatch of the run, including bench.py's
500 ms settle phase (thousands of launches, the DVFS dip among them), so its
average is not the timed region's.  bench.py's timed region is the last
`--steps` dispatches of the step's kernel before the after-timing
per-direction pass, which uses the separate seal/open kernels (other names).
This tool reads the run's kernel trace and writes, in rocprofv3's
kernel_stats.csv columns, the statistics of the last N dispatches of every
kernel whose name contains SUBSTR, plus the time from the first of those
dispatches' start to the last one's end (the timed region on the GPU).

usage: kernel_window.py TRACE_DIR SUBSTR N OUT_CSV
"""
import csv
import glob
import os
import statistics
import sys


def main(trace_dir, substr, n, out_csv):
    rows = []
    for f in glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += [r for r in csv.DictReader(fh) if substr in r["Kernel_Name"]]
    if not rows:
        raise SystemExit(f"no dispatch of {substr!r} under {trace_dir}")
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    by = {}
    for r in rows:
        by.setdefault(r["Kernel_Name"], []).append(r)
    name, disp = max(by.items(), key=lambda kv: len(kv[1]))
    last = disp[-n:]
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in last]
    span = int(last[-1]["End_Timestamp"]) - int(last[0]["Start_Timestamp"])
    with open(out_csv, "w", newline="") as fh:
        w = csv.writer(fh, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev",
                    "WindowSpanNs", "AllCallsInRun", "AllCallsAverageNs"])
        alld = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in disp]
        w.writerow([name, len(last), sum(d), sum(d) / len(d), 100.0, min(d), max(d),
                    statistics.pstdev(d), span, len(disp), sum(alld) / len(alld)])
    print(f"{name}: last {len(last)} of {len(disp)} dispatches avg {sum(d) / len(d) / 1e3:.2f} us "
          f"(all {sum(alld) / len(alld) / 1e3:.2f} us), span {span / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4])
