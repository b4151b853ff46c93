"""Per-kernel SQ/LDS counter summary of tools/gpu/pmc_sq.sh output:
VALU instructions per wave, VALU-busy share and LDS conflict cycles.
Usage: pmc_sq_report.py gpurun_out/pmcsq_<cfg> [kernel-substring]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if flt in r["Kernel_Name"]:
            agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in agg.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    waves = m.get("SQ_WAVES", 0) or 1
    line = [k]
    if "SQ_INSTS_VALU" in m:
        line.append(f"valu/wave {m['SQ_INSTS_VALU'] / waves:.0f}")
        line.append(f"lds/wave {m.get('SQ_INSTS_LDS', 0) / waves:.0f}")
    if "SQ_BUSY_CYCLES" in m and "SQ_ACTIVE_INST_VALU" in m:
        # SQ_BUSY_CYCLES summed over 32 SEs; ACTIVE_INST_VALU in quad-cycles over 1024 SIMDs
        busy = m["SQ_BUSY_CYCLES"] / 32
        valu = m["SQ_ACTIVE_INST_VALU"] * 4 / 1024
        line.append(f"busy {busy:.0f} cyc, valu-busy {valu / busy:.0%}")
    if "SQ_LDS_BANK_CONFLICT" in m:
        line.append(f"lds-conflict/CU {m['SQ_LDS_BANK_CONFLICT'] / 256:.0f} cyc, "
                    f"lds-active/CU {m.get('SQ_ACTIVE_INST_LDS', 0) / 256:.0f}")
    print(" | ".join(line))
