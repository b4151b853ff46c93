"""Per-kernel resource summary from a hipcc --cuda-device-only -S listing
(AMDGPU metadata): VGPRs, AGPRs, spills, LDS, scratch.  Usage: kinfo.py FILE.s [filter]"""
import re
import sys

text = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
meta = text[text.find("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    def g(key):
        m = re.search(r"\.%s:\s+(\S+)" % re.escape(key), blk)
        return m.group(1) if m else "?"
    name = g("name")
    if flt not in name:
        continue
    print(f"{name[:64]:64s} vgpr {g('vgpr_count'):>4} spill {g('vgpr_spill_count'):>3} "
          f"lds {g('group_segment_fixed_size'):>6} scratch {g('private_segment_fixed_size'):>4}")
