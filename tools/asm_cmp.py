#!/usr/bin/env python3
"""Per-function comparison of two gfx950 assembly listings (hipcc -S).

Round 6 (tools/ab/README.md): the A/B arms left the kernel sources, and every
kernel had to assemble to the same instructions as before.  This reads each
function body (from its `_Z...:` label to `.Lfunc_endN:`), drops comments,
.loc / .cfi lines and renumbers local labels, then reports per file how many
functions are identical, differ, disappeared or appeared.

usage: asm_cmp.py BEFORE_DIR AFTER_DIR NAME...   (NAME.s in both dirs)
  e.g. for f in aead_api launch_chacha launch_aes worker; do
         hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Iinclude -Inoise-c_amd/csrc \
               --cuda-device-only -S noise-c_amd/csrc/$f.hip -o /tmp/after/$f.s; done
"""
import re
import sys


def funcs(path):
    out, cur, body = {}, None, []
    for line in open(path):
        m = re.match(r'^(_Z\S+):\s*(;.*)?$', line)
        if m:
            cur, body = m.group(1), []
            continue
        if cur and re.match(r'^\.Lfunc_end\d+:', line):
            out[cur] = body
            cur = None
            continue
        if cur:
            t = line.split(';')[0].strip()
            if not t or t.startswith('.loc') or t.startswith('.cfi'):
                continue
            t = re.sub(r'\.LBB\d+_\d+', 'BB', t)
            t = re.sub(r'\.Ltmp\d+', 'TMP', t)
            body.append(t)
    return out


def main(before, after, names):
    bad = 0
    for f in names:
        a, b = funcs(f"{before}/{f}.s"), funcs(f"{after}/{f}.s")
        diff = [k for k in a if k in b and a[k] != b[k]]
        same = [k for k in a if k in b and a[k] == b[k]]
        gone, new = sorted(set(a) - set(b)), sorted(set(b) - set(a))
        print(f, "same", len(same), "differ", len(diff), "removed", len(gone), "new", len(new))
        for k in diff:
            print("  DIFF", k[:120])
        for k in gone:
            print("  GONE", k[:120])
        for k in new:
            print("  NEW", k[:120])
        bad += len(diff)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2], sys.argv[3:]))
