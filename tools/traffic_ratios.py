"""Every HBM-traffic ratio DESIGN.md §9 quotes, recomputed from the committed
PMC profiles (profiles/traffic_<cfg>.json: hbm_bytes_per_launch, the gfx950
FETCH_SIZE-corrected (2 FETCH + WRITE) bytes) over each kernel's algorithmic
bytes per launch (as bench.py counts them: input + output +
16-B tag per record, AD read, 40 B of key context per state; a duplex launch
is one seal and one open).  CPU only:

    python tools/traffic_ratios.py            # the table
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

def uniform_alg(cfg, duplex):
    import bench
    c = bench.CONFIGS[cfg]
    N, L, AD = c["records"], c["len"], c.get("ad", 0)
    S = c["states"]
    seal = N * (2 * L + 16 + AD) + S * 40
    return 2 * seal if duplex else seal


def c5_alg():
    """per cipher half of the C5 shard on rank 0: (records, payload bytes, states)"""
    import numpy as np
    import bench
    c = bench.CONFIGS["c5"]
    lay = bench.mixed_layout(c["records"], c["states"], 0)
    out = {}
    for name, parity in (("chacha", 0), ("aes", 1)):
        idx = np.nonzero((lay["st_global"] % 2) == parity)[0]
        states = len({int(s) for s in lay["st_global"][idx]})
        out[name] = 2 * int(lay["lens"][idx].sum()) + 16 * len(idx) + 40 * states
    return out


def main():
    rows = []
    for cfg in ("c2", "c3", "c4", "perf", "c5"):
        path = os.path.join(ROOT, "profiles", f"traffic_{cfg}.json")
        if not os.path.exists(path):
            continue
        ks = json.load(open(path))["kernels"]
        c5 = c5_alg() if cfg == "c5" else None
        for k, v in ks.items():
            hbm = v.get("hbm_bytes_per_launch")
            if not hbm or hbm < 5e6 or k.startswith(("at::", "gcm_prepare", "seg_plan")) or not k:
                continue
            if cfg == "c5":
                alg = c5["aes" if k.startswith("gcm") else "chacha"]
            else:
                alg = uniform_alg(cfg, "_duplex_" in k)
            rows.append((cfg, k, hbm / 1e6, alg / 1e6, hbm / alg))
    print(f"{'config':6} {'kernel':58} {'HBM MB':>9} {'alg MB':>9} {'ratio':>6}")
    for cfg, k, h, a, r in rows:
        print(f"{cfg:6} {k:58} {h:9.1f} {a:9.1f} {r:6.2f}")


if __name__ == "__main__":
    main()
