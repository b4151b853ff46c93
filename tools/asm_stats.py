#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc --cuda-device-only -S file.

usage: python tools/asm_stats.py FILE.s SYMBOL_SUBSTRING [--blocks]

Counts the kernel's instructions by class (VALU fast/slow as measured in
DESIGN.md §5, SALU, VMEM, LDS, branches) and, with --blocks, per basic block
(label), so the loop body of a kernel can be priced without a GPU.
"""
import re
import sys
from collections import Counter

FAST = re.compile(r"^v_(add_u32|sub_u32|subrev_u32|xor_b32|and_b32|or_b32|bitop3_b32|mov_b32|"
                  r"add_co_u32|addc_co_u32|sub_co_u32|subb_co_u32|cndmask_b32|not_b32)(_e32|_e64|_sdwa|_dpp)?$")


def klass(op: str) -> str:
    if op.startswith("v_"):
        if op.startswith(("v_cmp", "v_cmpx")):
            return "valu_cmp"
        return "valu_fast" if FAST.match(op) else "valu_slow"
    if op.startswith("s_waitcnt") or op in ("s_nop", "s_barrier", "s_setprio"):
        return "sync"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    blocks = "--blocks" in sys.argv
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        head = l.split(";")[0].rstrip()
        if l.startswith(("_Z", "__")) and head.endswith(":") and sym in head:
            start = i
            print("kernel:", head[:-1])
            break
    if start is None:
        raise SystemExit("symbol not found")
    tot, per, cur, ops = Counter(), {}, "entry", Counter()
    for l in lines[start + 1:]:
        if l.startswith("\t.end_amdhsa_kernel") or re.match(r"^\.Lfunc_end", l):
            break
        m = re.match(r"^(\.?[\w$.]+):", l)
        if m:
            cur = m.group(1)
            continue
        s = l.strip()
        if not s or s.startswith((".", ";", "//")):
            continue
        op = s.split()[0]
        k = klass(op)
        tot[k] += 1
        ops[op] += 1
        per.setdefault(cur, Counter())[k] += 1
    print("total:", dict(tot), "valu:", tot["valu_fast"] + tot["valu_slow"] + tot["valu_cmp"])
    if blocks:
        for b, c in per.items():
            v = c["valu_fast"] + c["valu_slow"] + c["valu_cmp"]
            if v >= 20:
                print(f"  {b:24s} valu {v:5d} (fast {c['valu_fast']}, slow {c['valu_slow']}) "
                      f"salu {c['salu']} vmem {c['vmem']} lds {c['lds']}")
    if "--ops" in sys.argv:
        for op, n in ops.most_common(40):
            print(f"    {op:28s} {n}")


if __name__ == "__main__":
    main()
