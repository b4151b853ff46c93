"""Summarise rocprofv3 --pmc CSV passes (tools/gpu/pmc.sh) per kernel and
write profiles/traffic_<config>.json for bench.py's roofline.traffic.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced stream
(double it); WRITE_SIZE reads exactly for 16-B/lane streaming stores.
Our loads are not all 16-B/lane-coalesced, so both the raw and the corrected
read figure are recorded (the correction is exact only for that pattern)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    """Kernel name without namespace/arguments, template args kept:
    'void na::gcm_staged<false>(na::UniformArgs)' -> 'gcm_staged<false>'."""
    n = name.split("(")[0].replace("void ", "").replace("na::", "").strip()
    return n


def load(d):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                vals[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return vals


def main(pmc_dir, config, out_json):
    agg = defaultdict(dict)
    for sub in sorted(os.listdir(pmc_dir)):
        p = os.path.join(pmc_dir, sub)
        if not os.path.isdir(p):
            continue
        for k, counters in load(p).items():
            for c, v in counters.items():
                agg[k][c] = sum(v) / len(v)
    kernels = {}
    for k, c in agg.items():
        e = dict(c)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            raw = (c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
            corr = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
            e["hbm_bytes_raw_per_launch"] = raw
            e["hbm_bytes_per_launch"] = corr
        kernels[k] = e
    out = {"config": config, "source": pmc_dir,
           "note": "per-launch averages; hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE) KiB "
                   "(gfx950 FETCH_SIZE half-count correction, MI355X_MICROARCH.md §HBM)",
           "kernels": kernels}
    with open(out_json, "w") as f:
        json.dump(out, f, indent=1)
    for k, e in kernels.items():
        print(k, {x: round(y, 1) for x, y in e.items()})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
