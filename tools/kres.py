#!/usr/bin/env python3
"""Register / scratch / occupancy / LDS report of the library's kernels,
from hipcc's kernel-resource-usage remarks (no GPU needed).
usage: python tools/kres.py [name-filter-regex]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-I../include",
       "-Icsrc", "-c", "csrc/aead_api.hip", "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, cwd=os.path.join(ROOT, "noise-c_amd"), capture_output=True, text=True).stderr
flt = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
cur, rows = None, {}
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*)", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].split(" [")[0].strip()
        rows[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1)
        rows[cur][k.strip()] = v.split("[")[0].strip()
for n, r in rows.items():
    if flt and not flt.search(n):
        continue
    g = lambda k: r.get(k, "?")
    print(f"{n[:70]:70s} vgpr {g('VGPRs'):>4s} scratch {g('ScratchSize [bytes/lane]'):>4s} "
          f"occ {g('Occupancy [waves/SIMD]')} lds {g('LDS Size [bytes/block]')}")
